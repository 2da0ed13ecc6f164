#!/bin/bash
# Quick GPU check of the working tree (GPU box): the GPU suite (optional), then bench lines.
# Usage: bash tools/gpu_quick.sh <tag> [suite] [workloads...]   e.g. gpu_quick.sh r05a suite cfg2 cfg4 bloom s125000
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=$1; shift; out=gpurun_out/$tag; mkdir -p $out
if [ "$1" = suite ]; then
  shift
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { tail -40 $out/pytest_gpu.log; exit 1; }
  tail -1 $out/pytest_gpu.log
fi
for wl in "$@"; do
  case $wl in
    s*) a="--strings ${wl#s} --steps 40 --warmup 5 --no-cpu-baseline" ;;
    cfg2) a="--steps 20 --warmup 3 --no-cpu-baseline" ;;
    *) a="--workload $wl --steps 10 --warmup 3 --no-cpu-baseline" ;;
  esac
  timeout -k 10 400 python -u bench.py $a > $out/bench_$wl.log 2>&1 || { tail -20 $out/bench_$wl.log; exit 1; }
  tail -1 $out/bench_$wl.log > $out/bench_$wl.json
  python3 -c "import json; d=json.loads(open('$out/bench_$wl.json').read()); print('$wl', '%.2f GB/s' % (d['value']/1e9), 'ms/step %.4f' % d['ms_per_step'], 'exact', d['exact_match']['rate'], d['exact_match']['sample'], 'tok ms %.4f' % d['stage_ms_per_step']['tokenize'])"
done
