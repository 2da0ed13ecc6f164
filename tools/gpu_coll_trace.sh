#!/bin/bash
# Kernel traces of the 125k-string step with and without the per-step all-reduce (DPT_BENCH_COLL=1
# forces the RCCL async path at world size 1).  Usage: bash tools/gpu_coll_trace.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/$1; mkdir -p $out
for c in 0 1; do
  DPT_BENCH_COLL=$c MASTER_ADDR=127.0.0.1 MASTER_PORT=2967$c timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/c$c -o run --output-format csv -- python3 bench.py --strings 125000 --steps 20 --warmup 3 --no-cpu-baseline --exact-sample 16384 > $out/c$c.log 2>&1 || { tail -20 $out/c$c.log; exit 1; }
  grep '^{' $out/c$c.log | tail -1 | cut -c1-160
  cut -c1-140 $out/c$c/run_kernel_stats.csv | head -14
done
