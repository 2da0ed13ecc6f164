#!/bin/bash
# GPU suite at the working tree, then the claim-policy A/B (tools/gpu_ab_tok.sh) and the phase
# diagnostic of the new default.  Usage: bash tools/gpu_claim_ab.sh <tag> lib1 lib2 ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=$1; shift; out=gpurun_out/$tag; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { tail -40 $out/pytest_gpu.log; exit 1; }
tail -2 $out/pytest_gpu.log
bash tools/gpu_ab_tok.sh $tag/ab "$@"
