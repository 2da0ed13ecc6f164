#!/bin/bash
# round 3: L2 prefetch of continuing strings' next windows (PF_NEXT) A/B; C2 sub-phase stops
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
B=dp-tokenization_amd/csrc/build
for wl in cfg4 cfg2; do
  bash tools/ab_libs_wl.sh $wl dp-tokenization_amd/dptok/libdpt.so $B/var_pf1/libdpt.so $B/var_pf2/libdpt.so $B/var_stop3/libdpt.so $B/var_c2s1/libdpt.so $B/var_c2s2/libdpt.so || exit 1
done
