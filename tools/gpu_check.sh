#!/bin/bash
# One GPU session: smoke, GPU parity tests, PMC traffic passes, the bench line, and a
# rocprofv3 kernel-trace summary of the bench.  Every GPU step has its own time limit and the
# chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=${STEPS:-10}
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 900 python tools/pmc_traffic.py 1000000 traffic > gpurun_out/pmc_traffic.log 2>&1 && \
cp profiles/pmc_traffic.json gpurun_out/pmc_traffic.json && \
timeout -k 10 600 python bench.py --steps $STEPS --warmup 3 > gpurun_out/bench.log 2>&1 && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof.log 2>&1
rc=$?
tail -3 gpurun_out/smoke.log gpurun_out/pytest_gpu.log gpurun_out/pmc_traffic.log gpurun_out/bench.log 2>/dev/null
exit $rc
