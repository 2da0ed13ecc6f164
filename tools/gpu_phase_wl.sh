#!/bin/bash
# Diagnostic: cumulative cost of the tokenize kernel's phases on a workload.  Builds stopped after a
# phase (make variant V=stopK DEFS=-DDPT_STOP=K; wrong results by design) timed by the rocprof kernel
# trace + one PMC pass each, next to the full build; then the s_memtime stamps build.
# Usage: bash tools/gpu_phase_wl.sh <tag> <N> <gen: ascii|s2orc|arabic> lib1 lib2 ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/$1; N=$2; GEN=$3; shift 3; mkdir -p $out
[ "$GEN" != ascii ] && { timeout -k 10 300 python3 tools/prof_driver.py $N 1 $GEN gen-only || exit 1; }
CTRS="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES"
for lib in "$@"; do
  tag=$(basename $(dirname $lib))
  DPT_LIB=$PWD/$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $out/$tag/trace -o run --output-format csv -- python3 tools/prof_driver.py $N 4 $GEN > $out/$tag.trace.log 2>&1 || { tail -5 $out/$tag.trace.log; exit 1; }
  DPT_LIB=$PWD/$lib timeout -k 10 120 rocprofv3 --kernel-trace --pmc $CTRS -d $out/$tag/p1 -o run --output-format csv -- python3 tools/prof_driver.py $N 2 $GEN > $out/$tag.pmc.log 2>&1 || { tail -5 $out/$tag.pmc.log; exit 1; }
  if [ "${PHASE_FETCH:-0}" = 1 ]; then   # HBM read bytes per stop build: where the reads beyond the input come from
    DPT_LIB=$PWD/$lib timeout -k 10 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $out/$tag/p2 -o run --output-format csv -- python3 tools/prof_driver.py $N 2 $GEN > $out/$tag.fetch.log 2>&1 || { tail -5 $out/$tag.fetch.log; exit 1; }
  fi
  echo "== $tag"
  python3 tools/pmc_summary.py $out/$tag | grep -A12 "kernel<256"
done
if [ -f dp-tokenization_amd/csrc/build/libdpt_stamps.so ] && [ "$GEN" != bloom ]; then
  timeout -k 10 120 python3 tools/stamps.py $N 256 $GEN > $out/stamps.log 2>&1 || { tail -5 $out/stamps.log; exit 1; }
  cat $out/stamps.log
fi
