#!/bin/bash
# round 3: token hash with an independent fingerprint state (the BLOOM-scale table now builds) +
# A_PREF (the generic walker reads the next atom before the trie load returns): GPU suite, A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/round_r03z; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { tail -40 $out/pytest_gpu.log; exit 1; }
tail -1 $out/pytest_gpu.log
B=dp-tokenization_amd/csrc/build
H=dp-tokenization_amd/dptok/libdpt.so
for r in 1 2; do
  bash tools/ab_libs_wl.sh bloom $H $B/var_apref0/libdpt.so || exit 1
  bash tools/ab_libs_wl.sh cfg5 $H $B/var_apref0/libdpt.so || exit 1
  bash tools/ab_libs_wl.sh cfg4 $H $B/var_apref0/libdpt.so || exit 1
done
bash tools/ab_libs_wl.sh cfg2 $H $B/var_apref0/libdpt.so || exit 1
