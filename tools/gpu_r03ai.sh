#!/bin/bash
# round 3: resident waves per CU at the strong-scaling shard sizes (DPT_WAVES_PER_CU 16 / 14 vs the default
# rule: ~7 strings per slot, 18 at 125k) + the fold-sequence test
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_fold.py -q -m gpu --timeout 200 --timeout-method thread 2>&1 | tail -1
for rep in 1 2; do
  for n in 125000 250000; do
    for w in 0 16 14; do
      DPT_WAVES_PER_CU=$w timeout -k 10 300 python3 bench.py --strings $n --steps 60 --warmup 5 --no-cpu-baseline --exact-sample 16384 > gpurun_out/w.log 2>&1 || { tail -5 gpurun_out/w.log; exit 1; }
      grep '^{' gpurun_out/w.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('%d wpc %-3s n %-8d GB/s %6.2f ms/step %.4f tokenize %.4f exact %s' % ($rep, '$w', $n, d['value']/1e9, d['ms_per_step'], d['stage_ms_per_step']['tokenize'], d['exact_match']['rate']))"
    done
  done
done
