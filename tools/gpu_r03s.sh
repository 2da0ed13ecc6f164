#!/bin/bash
# round 3: C2 id stores unconditional (masked-off lanes into a sink) vs the previous commit
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r03s
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r03s/pytest.log 2>&1 || { tail -40 gpurun_out/r03s/pytest.log; exit 1; }
tail -1 gpurun_out/r03s/pytest.log
B=dp-tokenization_amd/csrc/build
for wl in cfg4 cfg2 cfg5; do
  bash tools/ab_libs_wl.sh $wl dp-tokenization_amd/dptok/libdpt.so $B/var_prev/libdpt.so || exit 1
done
