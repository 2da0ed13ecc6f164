#!/bin/bash
# round 3: host path after the C list conversion (dptok/_pylists): drop-in GPU tests + --host-path line
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r03o
timeout -k 10 400 python -u -m pytest tests/test_llama_sp.py tests/test_compat.py tests/test_csr_lists.py -m "gpu or not gpu" -x -q --timeout 200 --timeout-method thread > gpurun_out/r03o/pytest.log 2>&1 || { tail -40 gpurun_out/r03o/pytest.log; exit 1; }
tail -1 gpurun_out/r03o/pytest.log
timeout -k 10 400 python -u bench.py --host-path > gpurun_out/r03o/host.log 2>&1 || { tail -20 gpurun_out/r03o/host.log; exit 1; }
tail -1 gpurun_out/r03o/host.log
