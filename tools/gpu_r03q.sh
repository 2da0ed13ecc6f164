#!/bin/bash
# round 3: timestamps on the dispatches + overwrite histogram (no per-step memset): GPU suite, then the
# strong-scaling points and cfg2
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r03q
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r03q/pytest.log 2>&1 || { tail -40 gpurun_out/r03q/pytest.log; exit 1; }
tail -1 gpurun_out/r03q/pytest.log
for n in 125000 250000 500000 1000000; do
  timeout -k 10 300 python -u bench.py --strings $n --steps 40 --warmup 5 --no-cpu-baseline --exact-sample 65536 > gpurun_out/r03q/strong_$n.log 2>&1 || { tail -20 gpurun_out/r03q/strong_$n.log; exit 1; }
  tail -1 gpurun_out/r03q/strong_$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print($n, '%.2f GB/s' % (d['value']/1e9), 'ms/step %.4f' % d['ms_per_step'], 'tok %.4f' % d['stage_ms_per_step']['tokenize'], 'exact', d['exact_match']['rate'])"
done
