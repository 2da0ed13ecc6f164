#!/bin/bash
# round 3: PUSH32 (forward_lanes64 span masks walked as 32-bit halves; var_push32 = 1, head = 0) A/B on BLOOM + the 64-lane tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
B=dp-tokenization_amd/csrc/build
H=dp-tokenization_amd/dptok/libdpt.so
DPT_LIB=$PWD/$B/var_push32/libdpt.so timeout -k 10 400 python -u -m pytest tests/test_bloom_scale.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread 2>&1 | tail -1
for r in 1 2; do
  bash tools/ab_libs_wl.sh bloom $H $B/var_push32/libdpt.so || exit 1
done
