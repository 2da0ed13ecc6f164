#!/bin/bash
# Marginal phase costs (DPT_DOUBLE variants) + per-phase stamps on cfg2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
B=dp-tokenization_amd/csrc/build
bash tools/ab_libs.sh dp-tokenization_amd/dptok/libdpt.so $(for k in ${DBL:-1 3 4 5}; do echo $B/var_dbl$k/libdpt.so; done) || exit 1
for g in ascii s2orc; do timeout -k 10 120 python tools/stamps.py 200000 256 $g || exit 1; done
