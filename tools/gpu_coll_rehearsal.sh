#!/bin/bash
# Rehearsal of bench.py's overlapped per-step all-reduce on a one-GPU box: the default line, the RCCL
# async path forced at world size 1 (DPT_BENCH_COLL=1, torch.distributed.run --nproc-per-node 1), and
# two gloo ranks sharing the card.  Usage: bash tools/gpu_coll_rehearsal.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/$1; mkdir -p $out
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --exact-sample 65536 > $out/plain.log 2>&1 || { tail -20 $out/plain.log; exit 1; }
tail -1 $out/plain.log | cut -c1-200
DPT_BENCH_COLL=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29612 \
    bench.py --steps 20 --warmup 5 --no-cpu-baseline --exact-sample 65536 > $out/rccl1.log 2>&1 || { tail -30 $out/rccl1.log; exit 1; }
grep '^{' $out/rccl1.log | tail -1 | cut -c1-200
DPT_BENCH_COLL=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29613 \
    bench.py --strings 125000 --steps 40 --warmup 5 --no-cpu-baseline --exact-sample 65536 > $out/rccl1_125k.log 2>&1 || { tail -30 $out/rccl1_125k.log; exit 1; }
grep '^{' $out/rccl1_125k.log | tail -1 | cut -c1-200
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29614 \
    bench.py --gpus 2 --steps 10 --warmup 3 --no-cpu-baseline --dist-backend gloo --exact-sample 65536 > $out/gloo2.log 2>&1 || { tail -30 $out/gloo2.log; exit 1; }
grep '^{' $out/gloo2.log | tail -1 | cut -c1-300
