#!/bin/bash
# Diagnostic: cumulative cost of the tokenize kernel's phases at HEAD.  Builds stopped after a phase
# (make variant V=stopK DEFS=-DDPT_STOP=K: 1 prep, 2 +A, 3 +B/C1; wrong results by design) are timed
# by the rocprof kernel trace and counted by one PMC pass each, next to the full build; then the
# s_memtime stamps build (make stamps) gives per-phase wave-time shares.
# Usage: bash tools/gpu_phase_diag.sh <tag> lib1 lib2 ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/$1; shift; mkdir -p $out
CTRS="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES"
for lib in "$@"; do
  tag=$(basename $(dirname $lib))
  DPT_LIB=$PWD/$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $out/$tag/trace -o run --output-format csv -- python3 tools/prof_driver.py 1000000 4 > $out/$tag.trace.log 2>&1 || { tail -5 $out/$tag.trace.log; exit 1; }
  DPT_LIB=$PWD/$lib timeout -k 10 120 rocprofv3 --kernel-trace --pmc $CTRS -d $out/$tag/p1 -o run --output-format csv -- python3 tools/prof_driver.py 1000000 2 > $out/$tag.pmc.log 2>&1 || { tail -5 $out/$tag.pmc.log; exit 1; }
  echo "== $tag"
  python3 tools/pmc_summary.py $out/$tag | grep -A12 "256, 16"
done
if [ -f dp-tokenization_amd/csrc/build/libdpt_stamps.so ]; then
  timeout -k 10 120 python3 tools/stamps.py 1000000 > $out/stamps.log 2>&1 || { tail -5 $out/stamps.log; exit 1; }
  cat $out/stamps.log
fi
