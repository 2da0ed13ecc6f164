#!/bin/bash
# round 3: the small-call resident-wave rule (~7 strings per slot) against the occupancy limit (DPT_NO_SMALL_WPC=1)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for rep in 1 2; do
  for n in 125000 250000; do
    for w in rule full; do
      if [ $w = full ]; then export DPT_NO_SMALL_WPC=1; else unset DPT_NO_SMALL_WPC; fi
      timeout -k 10 300 python3 bench.py --strings $n --steps 60 --warmup 5 --no-cpu-baseline --exact-sample 16384 > gpurun_out/w.log 2>&1 || { tail -5 gpurun_out/w.log; exit 1; }
      grep '^{' gpurun_out/w.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('%d %-4s n %-8d GB/s %6.2f ms/step %.4f tokenize %.4f exact %s' % ($rep, '$w', $n, d['value']/1e9, d['ms_per_step'], d['stage_ms_per_step']['tokenize'], d['exact_match']['rate']))"
    done
  done
done
