#!/bin/bash
# 1-GPU points at the per-rank shard sizes of 2/4/8-way strong scaling (1M / 500k / 250k / 125k
# strings of cfg2) and a kernel trace at 125k.  Usage: bash tools/gpu_strong_points.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/$1; mkdir -p $out
for n in 1000000 500000 250000 125000; do
  timeout -k 10 300 python -u bench.py --strings $n --steps 40 --warmup 5 --no-cpu-baseline > $out/bench_$n.log 2>&1 || { tail -20 $out/bench_$n.log; exit 1; }
  tail -1 $out/bench_$n.log > $out/bench_$n.json
  python3 -c "import json; d=json.loads(open('$out/bench_$n.json').read()); print($n, '%.2f GB/s' % (d['value']/1e9), 'ms/step %.4f' % d['ms_per_step'], 'tokenize %.4f' % d['stage_ms_per_step']['tokenize'], 'exact', d['exact_match']['rate'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace125k -o run --output-format csv -- python3 bench.py --strings 125000 --steps 20 --warmup 3 --no-cpu-baseline > $out/trace125k.log 2>&1 || { tail -5 $out/trace125k.log; exit 1; }
cut -c1-150 $out/trace125k/run_kernel_stats.csv
