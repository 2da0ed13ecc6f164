#!/bin/bash
# round 3: the 64-lane kernel's rec[] as two arrays (REC_SOA: 6.8 -> 5.2 KB LDS per wave) and more
# resident waves (WPE64 7 / 8: <= 72 / 64 VGPRs): BLOOM A/B; GPU suite at head
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
B=dp-tokenization_amd/csrc/build
H=dp-tokenization_amd/dptok/libdpt.so
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread 2>&1 | tail -2
for r in 1 2; do
  bash tools/ab_libs_wl.sh bloom $H $B/var_soa0/libdpt.so $B/var_wpe64_7/libdpt.so $B/var_wpe64_8/libdpt.so || exit 1
done
