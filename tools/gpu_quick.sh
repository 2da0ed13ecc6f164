#!/bin/bash
# Quick GPU iteration: parity tests, bench without CPU baseline, phase stamps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench.log 2>&1 || exit 1
tail -1 gpurun_out/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('value GB/s', d['value']/1e9, 'exact', d['exact_match'], 'stages', d['stage_ms_per_step'])"
timeout -k 10 200 python tools/stamps.py 200000 256 ascii && timeout -k 10 200 python tools/stamps.py 5000 0 s2orc
