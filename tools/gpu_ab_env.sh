#!/bin/bash
# A/B of environment knobs on the bench workload, one process each: bash tools/gpu_ab_env.sh "TAG=ENV ..." ...
# e.g. bash tools/gpu_ab_env.sh "base=" "wide=DPT_WIDE_STAGING=1"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for spec in "$@"; do
  tag=${spec%%=*}; envs=${spec#*=}
  env $envs timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --exact-sample 65536 > gpurun_out/bench_env_$tag.log 2>&1 || { tail -5 gpurun_out/bench_env_$tag.log; exit 1; }
  tail -1 gpurun_out/bench_env_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', 'GB/s %.2f' % (d['value']/1e9), 'exact', d['exact_match']['rate'], 'stages', {k: round(v,3) for k,v in d['stage_ms_per_step'].items()})"
done
