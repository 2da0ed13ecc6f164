#!/bin/bash
# round 3: WPE64 (the 256-byte 64-lane kernel capped at 80 VGPRs: 24 waves per CU instead of 20) A/B on BLOOM
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
B=dp-tokenization_amd/csrc/build
H=dp-tokenization_amd/dptok/libdpt.so
timeout -k 10 300 python -u -m pytest tests/test_bloom_scale.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "hash or bloom" 2>&1 | tail -3
for r in 1 2; do
  bash tools/ab_libs_wl.sh bloom $H $B/var_wpe64_6/libdpt.so $B/var_aref64_8/libdpt.so $B/var_aref64_1/libdpt.so $B/var_aslot8/libdpt.so || exit 1
done
# C2_NL: one-atom newline tokens resolved from the hash header (head) vs the walkers (var_c2nl0)
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread 2>&1 | tail -2
for r in 1 2; do
  bash tools/ab_libs_wl.sh cfg4 $H $B/var_c2nl0/libdpt.so || exit 1
  bash tools/ab_libs_wl.sh cfg5 $H $B/var_c2nl0/libdpt.so || exit 1
done
bash tools/ab_libs_wl.sh cfg2 $H $B/var_c2nl0/libdpt.so || exit 1
