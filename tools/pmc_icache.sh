#!/bin/bash
# Instruction-fetch PMC pass (instruction cache requests / misses, fetches, branches) on cfg2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/pmc_icache; mkdir -p $out
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQC_ICACHE_REQ SQC_ICACHE_MISSES SQ_IFETCH SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_INST_CYCLES_SALU SQ_WAVES SQ_BUSY_CYCLES -d $out/p1 -o run --output-format csv -- python3 tools/prof_driver.py 1000000 2 ascii > $out/p1.log 2>&1 || { tail -5 $out/p1.log; exit 1; }
python3 tools/pmc_summary.py $out | grep -A9 "256, 16, false, false"
