#!/bin/bash
# PMC comparison of libdpt.so builds on cfg2 (1M strings): instruction counts and the memory
# pipeline's busy cycles, one rocprofv3 pass per counter group.  Usage: bash tools/gpu_pmc_ab.sh <tag> lib1 lib2 ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/$1; shift; mkdir -p $out
for lib in "$@"; do
  tag=$(basename $(dirname $lib))
  i=0
  for set in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES" \
             "TA_TA_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCC_HIT_sum TCC_MISS_sum"; do
    i=$((i+1))
    DPT_LIB=$PWD/$lib timeout -k 10 120 rocprofv3 --kernel-trace --pmc $set -d $out/$tag/p$i -o run --output-format csv -- python3 tools/prof_driver.py 1000000 2 > $out/$tag.p$i.log 2>&1 || { tail -5 $out/$tag.p$i.log; exit 1; }
  done
  DPT_LIB=$PWD/$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $out/$tag/trace -o run --output-format csv -- python3 tools/prof_driver.py 1000000 4 > $out/$tag.trace.log 2>&1 || { tail -5 $out/$tag.trace.log; exit 1; }
  echo "== $tag"
  python3 tools/pmc_summary.py $out/$tag | grep -A14 "256, 16"
done
