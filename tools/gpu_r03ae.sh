#!/bin/bash
# round 3: forward_lanes64's long chunks through the row recurrence (LANES64_ROW_T; head = 16): GPU suite, BLOOM A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
B=dp-tokenization_amd/csrc/build
H=dp-tokenization_amd/dptok/libdpt.so
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread 2>&1 | tail -2
for r in 1 2; do
  bash tools/ab_libs_wl.sh bloom $H $B/var_rowt8/libdpt.so $B/var_rowt32/libdpt.so $B/var_rowt1000/libdpt.so || exit 1
done
