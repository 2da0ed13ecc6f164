#!/bin/bash
# round 3: per-phase wave residency (s_memtime stamps build), C2 split into bulk / hash / pending+walkers
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python tools/stamps.py 1000000 256 ascii > gpurun_out/stamps_cfg2.log 2>&1 || { tail -20 gpurun_out/stamps_cfg2.log; exit 1; }
timeout -k 10 300 python tools/stamps.py 200000 0 s2orc > gpurun_out/stamps_cfg4.log 2>&1 || { tail -20 gpurun_out/stamps_cfg4.log; exit 1; }
cat gpurun_out/stamps_cfg2.log gpurun_out/stamps_cfg4.log
