#!/bin/bash
# A/B: batch sums by tokenize-side atomics + one-block scan (the product build) vs HEAD's look-back
# finish, and the pending-row capacity (PEND_CAP 64 / 32 / 16): GPU suite on the product build, then
# per lib the finish A/B lines (1M and 125k strings) and the tokenize kernel's HBM traffic.
# Usage: bash tools/gpu_ab_pend.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=$1; out=gpurun_out/$tag; mkdir -p $out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { tail -30 $out/pytest_gpu.log; exit 1; }
tail -1 $out/pytest_gpu.log
C=dp-tokenization_amd/csrc/build
bash tools/gpu_ab_fin.sh $tag/fin $C/var_head/libdpt.so dp-tokenization_amd/dptok/libdpt.so $C/var_p32/libdpt.so $C/var_p16/libdpt.so || exit 1
for v in var_head var_p32 var_p16; do
  DPT_LIB=$PWD/$C/$v/libdpt.so timeout -k 10 300 python3 tools/pmc_traffic.py 1000000 ${tag}_$v > $out/traffic_$v.log 2>&1 || { tail -5 $out/traffic_$v.log; exit 1; }
  echo $v; tail -1 $out/traffic_$v.log | cut -c1-400
done
