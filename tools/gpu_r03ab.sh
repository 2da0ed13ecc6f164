#!/bin/bash
# round 3: A_SLOT8 on top of WPE64=6 (head = both), then the final evidence session (tools/gpu_round3c.sh r03ab)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
B=dp-tokenization_amd/csrc/build
H=dp-tokenization_amd/dptok/libdpt.so
for r in 1 2; do
  bash tools/ab_libs_wl.sh bloom $H $B/var_aslot8_0/libdpt.so || exit 1
done
bash tools/gpu_round3c.sh r03ab
