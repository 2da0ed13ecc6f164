#!/bin/bash
# round 3: marginal phase costs in the full kernel (each phase run twice: DPT_DOUBLE builds)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
B=dp-tokenization_amd/csrc/build
for wl in cfg2 cfg4; do
  bash tools/ab_libs_wl.sh $wl dp-tokenization_amd/dptok/libdpt.so $B/var_dbl5/libdpt.so $B/var_dbl1/libdpt.so $B/var_dbl3/libdpt.so $B/var_dbl4/libdpt.so || exit 1
done
