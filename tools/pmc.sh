#!/bin/bash
# PMC passes (each its own rocprofv3 run, kernel-trace only -- no sys/runtime trace) on the
# device-path driver.  Usage: bash tools/pmc.sh <tag> [N] [gen]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=$1; N=${2:-1000000}; GEN=${3:-ascii}
out=gpurun_out/pmc_$tag; mkdir -p $out
[ "$GEN" != ascii ] && { timeout -k 10 300 python3 tools/prof_driver.py $N 1 $GEN gen-only || exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace -o run --output-format csv -- python3 tools/prof_driver.py $N 3 $GEN > $out/trace.log 2>&1 || exit 1
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE" \
           "TA_TA_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCC_HIT_sum TCC_MISS_sum" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $set -d $out/p$i -o run --output-format csv -- python3 tools/prof_driver.py $N 3 $GEN > $out/p$i.log 2>&1 || exit 1
done
python3 tools/pmc_summary.py $out > $out/summary.txt && cat $out/summary.txt
