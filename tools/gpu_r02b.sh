#!/bin/bash
# GPU suite, a quick cfg2 bench line, the host-path line, and a kernel trace of the 125k-string
# strong-scaling point (fixed costs per step).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/${1:-r02b}; mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { tail -40 $out/pytest_gpu.log; exit 1; }
tail -3 $out/pytest_gpu.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $out/bench.log 2>&1 || { tail -20 $out/bench.log; exit 1; }
tail -1 $out/bench.log | cut -c1-600
timeout -k 10 300 python -u bench.py --host-path > $out/host.log 2>&1 || { tail -20 $out/host.log; exit 1; }
tail -1 $out/host.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace125k -o run --output-format csv -- python3 bench.py --strings 125000 --steps 20 --warmup 5 --no-cpu-baseline > $out/trace125k.log 2>&1 || { tail -20 $out/trace125k.log; exit 1; }
find $out/trace125k -name "*kernel_stats.csv" | head -1 | xargs cat | cut -c1-160 | head -14
