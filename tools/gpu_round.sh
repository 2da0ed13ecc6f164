#!/bin/bash
TAG=${1:-v12}
# v12 evidence: smoke + GPU parity, the profile round (traffic, bench line, rocprof trace, PMC),
# and the cfg4 / cfg5 bench lines
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && \
bash tools/profile_round.sh $TAG > gpurun_out/round_$TAG.log 2>&1 && \
timeout -k 10 300 python bench.py --workload cfg4 --no-cpu-baseline > gpurun_out/bench_cfg4.log 2>&1 && \
timeout -k 10 300 python bench.py --workload cfg5 --no-cpu-baseline > gpurun_out/bench_cfg5.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_gpu.log; tail -15 gpurun_out/round_$TAG.log | cut -c1-400; tail -1 gpurun_out/bench_cfg4.log | cut -c1-200; tail -1 gpurun_out/bench_cfg5.log | cut -c1-200; exit $rc
