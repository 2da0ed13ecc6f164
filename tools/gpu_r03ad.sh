#!/bin/bash
# round 3: LANES64_ODD A/B on BLOOM; BLOOM phase table at HEAD (stop builds 1 / 2 / 26 / 3 + full)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
B=dp-tokenization_amd/csrc/build
H=dp-tokenization_amd/dptok/libdpt.so
for r in 1 2; do
  bash tools/ab_libs_wl.sh bloom $H $B/var_odd/libdpt.so || exit 1
done
bash tools/gpu_phase_wl.sh phase_bloom_r03ad 200000 bloom $B/var_stop1/libdpt.so $B/var_stop2/libdpt.so $B/var_stop26/libdpt.so $B/var_stop3/libdpt.so $H
