#!/bin/bash
# smoke, GPU parity tests, then an env A/B of the staging width and one default bench line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && \
bash tools/gpu_ab_env.sh "narrow=" "wide=DPT_WIDE_STAGING=1" "narrow2=" "wide2=DPT_WIDE_STAGING=1" > gpurun_out/ab.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_fullexact.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; cat gpurun_out/ab.log; tail -1 gpurun_out/bench_fullexact.log | cut -c1-300; exit $rc
