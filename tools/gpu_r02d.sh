#!/bin/bash
# Round-2 GPU session d: GPU suite, HBM traffic of the HEAD kernels (profiles/pmc_traffic.json), the
# PMC summary, the headline line with the CPU baseline, and a kernel trace of the bloom workload.
# Usage: bash tools/gpu_r02d.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=$1; out=gpurun_out/$tag; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { tail -40 $out/pytest_gpu.log; exit 1; }
tail -2 $out/pytest_gpu.log
timeout -k 10 600 python3 tools/pmc_traffic.py 1000000 $tag > $out/traffic.log 2>&1 || { tail -20 $out/traffic.log; exit 1; }
tail -1 $out/traffic.log
bash tools/pmc.sh $tag > $out/pmc.log 2>&1 || { tail -20 $out/pmc.log; exit 1; }
tail -30 $out/pmc.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $out/bench.log 2>&1 || { tail -20 $out/bench.log; exit 1; }
tail -1 $out/bench.log > $out/bench.json; cat $out/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 10 --warmup 3 > $out/trace.log 2>&1 || { tail -20 $out/trace.log; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $out/trace_bloom -o run --output-format csv -- python3 bench.py --workload bloom --gen-procs 1 --strings 200000 --steps 10 --warmup 3 --no-cpu-baseline --exact-sample 20000 > $out/trace_bloom.log 2>&1 || { tail -20 $out/trace_bloom.log; exit 1; }
for d in trace trace_bloom; do find $out/$d -name "*kernel_stats.csv" | head -1 | xargs cat | cut -c1-150 | head -8; done
