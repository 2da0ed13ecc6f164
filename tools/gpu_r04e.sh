#!/bin/bash
# round 4: which kernel the self-copy's slow calls spend their time in (kernel trace, 125k cfg2)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/r04e; mkdir -p $out
DPT_SELF_COPY=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o sc1 -- python3 bench.py --workload cfg2 --strings 125000 --steps 3 --warmup 1 --no-cpu-baseline --exact-sample 4096 > $out/bench_sc1.log 2>&1 || { tail -5 $out/bench_sc1.log; exit 1; }
tail -1 $out/bench_sc1.log | cut -c1-300
f=$(find $out/prof -name '*kernel_stats.csv' | head -1); cut -c1-200 $f | head -12
