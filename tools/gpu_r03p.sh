#!/bin/bash
# round 3: kernel trace of the 125k strong-scaling point (per-kernel times and the gaps between them)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r03p
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03p/prof -o run -- python3 bench.py --strings 125000 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r03p/bench.log 2>&1 || { tail -20 gpurun_out/r03p/bench.log; exit 1; }
tail -1 gpurun_out/r03p/bench.log
find gpurun_out/r03p/prof -name "*kernel_stats.csv" -exec cat {} \;
