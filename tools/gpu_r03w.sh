#!/bin/bash
# round 3: BLOOM phase table after forward_lanes64 (stop builds 1 / 2 / 25 / 26 / 3 and the full build)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
B=dp-tokenization_amd/csrc/build
bash tools/gpu_phase_wl.sh phase_bloom_r03w 200000 bloom $B/var_stop25/libdpt.so $B/var_stop26/libdpt.so $B/var_stop3/libdpt.so dp-tokenization_amd/dptok/libdpt.so
