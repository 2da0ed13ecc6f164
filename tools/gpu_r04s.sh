#!/bin/bash
# round 4 at HEAD: kernel traces + stats of the 125k strong-scaling point and of cfg4
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/r04s; mkdir -p $out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/t125k -o run --output-format csv -- python3 bench.py --strings 125000 --steps 20 --warmup 3 --no-cpu-baseline --exact-sample 4096 > $out/t125k.log 2>&1 || { tail -5 $out/t125k.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/tcfg4 -o run --output-format csv -- python3 bench.py --workload cfg4 --steps 10 --warmup 3 --no-cpu-baseline --exact-sample 4096 > $out/tcfg4.log 2>&1 || { tail -5 $out/tcfg4.log; exit 1; }
for d in t125k tcfg4; do echo "== $d"; cut -c1-140 $(find $out/$d -name "*kernel_stats.csv" | head -1) | head -8; done
