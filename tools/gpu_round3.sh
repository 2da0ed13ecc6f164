#!/bin/bash
# Round-3 evidence, part 1 (GPU box): the GPU suite, HBM traffic (calibrated PMC passes), the default
# bench line (with the CPU baseline), its rocprofv3 kernel trace + stats, the PMC summary.
# Usage: bash tools/gpu_round3.sh <tag>  -> gpurun_out/round_<tag>/
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=$1; out=gpurun_out/round_$tag; mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { tail -40 $out/pytest_gpu.log; exit 1; }
tail -1 $out/pytest_gpu.log
timeout -k 10 600 python3 tools/pmc_traffic.py 1000000 $tag > $out/traffic.log 2>&1 || { tail -20 $out/traffic.log; exit 1; }
tail -1 $out/traffic.log
timeout -k 10 400 python -u bench.py > $out/bench.log 2>&1 || { tail -20 $out/bench.log; exit 1; }
tail -1 $out/bench.log > $out/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 10 --warmup 3 > $out/trace.log 2>&1 || { tail -20 $out/trace.log; exit 1; }
bash tools/pmc.sh $tag > $out/pmc.log 2>&1 || { tail -20 $out/pmc.log; exit 1; }
cat $out/bench.json
find $out/trace -name "*kernel_stats.csv" | head -1 | xargs cat | cut -c1-200 | head -12
