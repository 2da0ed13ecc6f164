#!/bin/bash
# A/B the resident waves per CU of the first-pass kernel (DPT_WAVES_PER_CU; "0" = occupancy API).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for w in ${WAVES:-0 4 7 10}; do
  DPT_WAVES_PER_CU=$w timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --exact-sample 16384 > gpurun_out/bench_w$w.log 2>&1 || { tail -5 gpurun_out/bench_w$w.log; exit 1; }
  tail -1 gpurun_out/bench_w$w.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('waves/CU $w', 'GB/s %.2f' % (d['value']/1e9), 'exact', d['exact_match']['rate'], 'tokenize ms %.2f' % d['stage_ms_per_step']['tokenize'])"
done
