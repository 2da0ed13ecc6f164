#!/bin/bash
# round 3: MachineLICM off for the kernels (no SGPR/VGPR spills), extra kernarg refresh points
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
B=dp-tokenization_amd/csrc/build
for wl in cfg2 cfg4 cfg5 bloom; do
  bash tools/ab_libs_wl.sh $wl dp-tokenization_amd/dptok/libdpt.so $B/var_licm0/libdpt.so $B/var_licm0km/libdpt.so $B/var_km/libdpt.so || exit 1
done
