#!/bin/bash
# Round-2 GPU session c: the GPU suite (incl. the BLOOM-scale tests), the headline line, the bloom
# workload line and a kernel trace of the bloom workload.  Usage: bash tools/gpu_r02c.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/$1; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { tail -40 $out/pytest_gpu.log; exit 1; }
tail -2 $out/pytest_gpu.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $out/bench_cfg2.log 2>&1 || { tail -20 $out/bench_cfg2.log; exit 1; }
tail -1 $out/bench_cfg2.log > $out/bench_cfg2.json
timeout -k 10 400 python -u bench.py --workload bloom --steps 20 --warmup 5 > $out/bench_bloom.log 2>&1 || { tail -20 $out/bench_bloom.log; exit 1; }
tail -1 $out/bench_bloom.log > $out/bench_bloom.json
for f in $out/bench_*.json; do
  python3 -c "import json,sys; d=json.loads(open('$f').read()); print('$f', '%.2f GB/s' % (d['value']/1e9), 'ms/step %.4f' % d['ms_per_step'], 'exact', d['exact_match']['rate'], d['exact_match']['sample'], 'tok ms %.4f' % d['stage_ms_per_step']['tokenize'], 'frac %.4f' % d['roofline']['frac'], 'cpu', d['cpu_baseline'])"
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/trace_bloom -o run --output-format csv -- python3 bench.py --workload bloom --steps 10 --warmup 3 --no-cpu-baseline --exact-sample 20000 > $out/trace_bloom.log 2>&1 || { tail -20 $out/trace_bloom.log; exit 1; }
find $out/trace_bloom -name "*kernel_stats.csv" | head -1 | xargs cat | cut -c1-150 | head -8
