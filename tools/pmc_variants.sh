#!/bin/bash
# One PMC pass (instruction mix + wait cycles) per library build: the base library and the
# DPT_DOUBLE variants, so a phase's instruction count = variant - base.  Usage: bash tools/pmc_variants.sh lib...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY"
for lib in "$@"; do
  tag=$(basename $(dirname $lib))
  out=gpurun_out/pmcv_$tag; mkdir -p $out
  DPT_LIB=$PWD/$lib timeout -k 10 120 rocprofv3 --kernel-trace --pmc $C -d $out/p1 -o run --output-format csv -- python3 tools/prof_driver.py 1000000 2 ascii > $out/p1.log 2>&1 || { tail -5 $out/p1.log; exit 1; }
  echo "== $tag"; python3 tools/pmc_summary.py $out | grep -A9 "256, 16, false, false"
done
