#!/bin/bash
# One GPU iteration: gpu parity tests (stop at first failure), then a short bench without the CPU leg.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
for w in ${WORKLOADS:-cfg2}; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_$w.log 2>&1 || { tail -20 gpurun_out/bench_$w.log; exit 1; }
  tail -1 gpurun_out/bench_$w.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$w GB/s %.2f' % (d['value']/1e9), 'exact', d['exact_match']['rate'], 'stages', {k: round(v,3) for k,v in d['stage_ms_per_step'].items()})"
  if [ -n "$AB" ]; then DPT_B=rows timeout -k 10 300 python -u bench.py --workload $w --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_${w}_rows.log 2>&1 && tail -1 gpurun_out/bench_${w}_rows.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$w DPT_B=rows GB/s %.2f' % (d['value']/1e9), d['exact_match']['rate'])" || exit 1; fi
done
