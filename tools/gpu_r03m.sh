#!/bin/bash
# round 3: exposed cost of C2's id stores (diagnostic builds without them: nost1 bulk, nost3 bulk + hash)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
B=dp-tokenization_amd/csrc/build
for wl in cfg4 cfg2; do
  bash tools/ab_libs_wl.sh $wl dp-tokenization_amd/dptok/libdpt.so $B/var_nost1/libdpt.so $B/var_nost3/libdpt.so || exit 1
done
