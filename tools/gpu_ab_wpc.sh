#!/bin/bash
# Resident waves per CU of the 16-lane first pass (DPT_WAVES_PER_CU) at the strong-scaling shard sizes:
# interleaved bench lines, no profiler.  Usage: bash tools/gpu_ab_wpc.sh <tag> "22 20 18 16"
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/$1; mkdir -p $out
for rep in 1 2; do
  for n in 125000 250000 500000 1000000; do
    for w in $2; do
      DPT_WAVES_PER_CU=$w timeout -k 10 300 python3 bench.py --strings $n --steps 20 --warmup 5 --no-cpu-baseline --exact-sample 16384 > $out/$w.$n.$rep.log 2>&1 || { tail -5 $out/$w.$n.$rep.log; exit 1; }
      grep '^{' $out/$w.$n.$rep.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('%d wpc %-3s n %-8d GB/s %6.2f ms/step %.4f tokenize %.4f exact %s' % ($rep, '$w', $n, d['value']/1e9, d['ms_per_step'], d['stage_ms_per_step']['tokenize'], d['exact_match']['rate']))"
    done
  done
done
