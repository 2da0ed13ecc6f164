#!/bin/bash
# round 4 at HEAD: (1) per-phase PMC of the 16-lane kernel -- LDS bank conflicts, waits, instructions --
# from the DPT_STOP / DPT_C2STOP builds of the HEAD source on cfg2 and cfg4 (tools/phase_table.py);
# (2) the BLOOM-scale 64-lane kernel's kernel trace + PMC summary; (3) the PUSH32 A/B on BLOOM.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
B=dp-tokenization_amd/csrc/build
H=dp-tokenization_amd/dptok/libdpt.so   # the product build
out=gpurun_out/r04l; mkdir -p $out/phase
CTRS="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VALU"
part=${1:-all}
if [ $part != 2 ]; then
timeout -k 10 300 python3 tools/prof_driver.py 200000 1 s2orc gen-only || exit 1
for wl in "ascii 1000000" "s2orc 200000"; do
  set -- $wl
  for lib in $B/var_stop1/libdpt.so $B/var_stop21/libdpt.so $B/var_stop2/libdpt.so $B/var_stop3/libdpt.so \
             $B/var_c2s1/libdpt.so $B/var_c2s2/libdpt.so $H; do
    tag=$(basename $(dirname $lib))_$1
    d=$out/phase/$tag
    DPT_LIB=$PWD/$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $d/trace -o run --output-format csv -- python3 tools/prof_driver.py $2 3 $1 > $d.trace.log 2>&1 || { tail -5 $d.trace.log; exit 1; }
    DPT_LIB=$PWD/$lib timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $CTRS -d $d/p1 -o run --output-format csv -- python3 tools/prof_driver.py $2 2 $1 > $d.pmc.log 2>&1 || { tail -5 $d.pmc.log; exit 1; }
    echo "== $tag"; python3 tools/pmc_summary.py $d | grep -A9 "256, 16" | head -10
  done
done
fi
[ $part = 1 ] && exit 0
# BLOOM scale: corpus, kernel trace + PMC passes (tools/pmc.sh)
timeout -k 10 600 python3 tools/prof_driver.py 500000 1 bloom gen-only || exit 1
timeout -k 10 900 bash tools/pmc.sh r04l_bloom 500000 bloom > $out/bloom_pmc.log 2>&1 || { tail -20 $out/bloom_pmc.log; exit 1; }
tail -40 $out/bloom_pmc.log
# PUSH32 A/B (BLOOM), twice, interleaved
for r in 1 2; do
  timeout -k 10 600 bash tools/ab_libs_wl.sh bloom $H $B/var_push32/libdpt.so || exit 1
done
