#!/bin/bash
# A/B the first-pass kernel variants on the bench workload (one process each; same GPU).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for v in ${VARIANTS:-lane rows16}; do
  DPT_KERNEL=$v timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --exact-sample 65536 > gpurun_out/bench_$v.log 2>&1 || { tail -5 gpurun_out/bench_$v.log; exit 1; }
  tail -1 gpurun_out/bench_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', 'GB/s %.2f' % (d['value']/1e9), 'exact', d['exact_match']['rate'], 'stages', {k: round(v,3) for k,v in d['stage_ms_per_step'].items()})"
done
