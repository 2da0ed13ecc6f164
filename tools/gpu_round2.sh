#!/bin/bash
# Round-2 GPU session: the GPU suite, the default bench line, the strong-scaling points (1-GPU runs at
# the per-rank shard of 2/4/8-way cfg3), the host-path line, and a kernel trace of the 125k point.
# Usage: bash tools/gpu_round2.sh <tag> [skip-tests]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/$1; mkdir -p $out
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { tail -40 $out/pytest_gpu.log; exit 1; }
  tail -2 $out/pytest_gpu.log
fi
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $out/bench_1m.log 2>&1 || { tail -20 $out/bench_1m.log; exit 1; }
tail -1 $out/bench_1m.log > $out/bench_1m.json
for n in 500000 250000 125000; do
  timeout -k 10 300 python -u bench.py --strings $n --steps 40 --warmup 5 --no-cpu-baseline > $out/bench_$n.log 2>&1 || { tail -20 $out/bench_$n.log; exit 1; }
  tail -1 $out/bench_$n.log > $out/bench_$n.json
done
for f in $out/bench_*.json; do
  python3 -c "import json,sys; d=json.loads(open('$f').read()); print('$f', '%.2f GB/s' % (d['value']/1e9), 'ms/step %.4f' % d['ms_per_step'], 'exact', d['exact_match']['rate'], d['exact_match']['sample'], 'tok ms %.4f' % d['stage_ms_per_step']['tokenize'], 'frac %.4f' % d['roofline']['frac'])"
done
if [ -n "$HOSTPATH" ]; then
  timeout -k 10 300 python -u bench.py --host-path > $out/host.log 2>&1 || { tail -20 $out/host.log; exit 1; }
  tail -1 $out/host.log
fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace125k -o run --output-format csv -- python3 bench.py --strings 125000 --steps 20 --warmup 5 --no-cpu-baseline > $out/trace125k.log 2>&1 || { tail -20 $out/trace125k.log; exit 1; }
find $out/trace125k -name "*kernel_stats.csv" | head -1 | xargs cat | cut -c1-140 | head -12
