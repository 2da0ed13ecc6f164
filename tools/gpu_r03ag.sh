#!/bin/bash
# round 3: cfg4 knob sweep on HEAD: A_REFILL 16 / 8 (16-lane kernel), WPE16 5
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
B=dp-tokenization_amd/csrc/build
H=dp-tokenization_amd/dptok/libdpt.so
for r in 1 2; do
  bash tools/ab_libs_wl.sh cfg4 $H $B/var_aref16/libdpt.so $B/var_aref8/libdpt.so $B/var_wpe16_5/libdpt.so || exit 1
done
bash tools/ab_libs_wl.sh cfg2 $H $B/var_aref16/libdpt.so $B/var_aref8/libdpt.so $B/var_wpe16_5/libdpt.so || exit 1
