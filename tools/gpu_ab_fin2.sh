#!/bin/bash
# Finish-pass A/B (split-batch finish vs HEAD's look-back): GPU suite on the product build, then
# tools/gpu_ab_fin.sh over HEAD's lib, the product lib and variants (1M and 125k strings).
# Usage: bash tools/gpu_ab_fin2.sh <tag> lib...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=$1; shift; out=gpurun_out/$tag; mkdir -p $out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { tail -30 $out/pytest_gpu.log; exit 1; }
tail -1 $out/pytest_gpu.log
bash tools/gpu_ab_fin.sh $tag/fin "$@"
