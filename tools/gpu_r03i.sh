#!/bin/bash
# round 3: walker select/defer + hash-pass rounds A/B (parity first)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r03i
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03i/pytest.log 2>&1 || { tail -40 gpurun_out/r03i/pytest.log; exit 1; }
tail -1 gpurun_out/r03i/pytest.log
B=dp-tokenization_amd/csrc/build
for wl in cfg2 cfg4; do
  bash tools/ab_libs_wl.sh $wl dp-tokenization_amd/dptok/libdpt.so $B/var_base/libdpt.so $B/var_asch0/libdpt.so $B/var_hpu1/libdpt.so $B/var_hpu4/libdpt.so || exit 1
done
