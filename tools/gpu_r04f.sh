#!/bin/bash
# round 4: per-phase stamps of the first pass with the self-copy on / off (libdpt_stamps.so), 125k cfg2
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/r04f; mkdir -p $out
for sc in 1 0; do
  DPT_SELF_COPY=$sc timeout -k 10 120 python3 tools/stamps.py ${N:-125000} > $out/stamps_sc$sc.txt 2>&1 || { tail -5 $out/stamps_sc$sc.txt; exit 1; }
  echo "sc=$sc"; cat $out/stamps_sc$sc.txt
done
