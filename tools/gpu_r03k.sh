#!/bin/bash
# round 3: ASCII walker one back edge + 32-bit newline expansion (head) vs two edges (oe0); L2 prefetch of
# continuing strings' next windows (PF_NEXT 1/2); C2 sub-phase stops (c2s1 bulk only, c2s2 + hash, stop3 no C2)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r03k
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03k/pytest.log 2>&1 || { tail -40 gpurun_out/r03k/pytest.log; exit 1; }
tail -1 gpurun_out/r03k/pytest.log
B=dp-tokenization_amd/csrc/build
for wl in cfg4 cfg2; do
  bash tools/ab_libs_wl.sh $wl dp-tokenization_amd/dptok/libdpt.so $B/var_oe0/libdpt.so $B/var_pf1/libdpt.so $B/var_pf2/libdpt.so $B/var_stop3/libdpt.so $B/var_c2s1/libdpt.so $B/var_c2s2/libdpt.so || exit 1
done
