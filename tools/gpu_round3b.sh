#!/bin/bash
# Round-3 evidence, part 2: the other workloads' lines, the strong-scaling points (1-GPU runs at the
# per-rank shard sizes of cfg3), the host-path line.  Usage: bash tools/gpu_round3b.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=$1; out=gpurun_out/round_$tag; mkdir -p $out
for wl in cfg1 cfg4 cfg5 bloom; do
  timeout -k 10 400 python -u bench.py --workload $wl --steps 10 --warmup 3 > $out/bench_$wl.log 2>&1 || { tail -20 $out/bench_$wl.log; exit 1; }
  tail -1 $out/bench_$wl.log > $out/bench_$wl.json
done
for n in 500000 250000 125000; do
  timeout -k 10 300 python -u bench.py --strings $n --steps 40 --warmup 5 --no-cpu-baseline > $out/strong_$n.log 2>&1 || { tail -20 $out/strong_$n.log; exit 1; }
  tail -1 $out/strong_$n.log > $out/strong_$n.json
done
timeout -k 10 400 python -u bench.py --host-path > $out/host.log 2>&1 || { tail -20 $out/host.log; exit 1; }
tail -1 $out/host.log > $out/host_path.json
for f in $out/bench_*.json $out/strong_*.json; do
  python3 -c "import json,sys; d=json.loads(open('$f').read()); print('$f', '%.2f GB/s' % (d['value']/1e9), 'ms/step %.4f' % d['ms_per_step'], 'exact', d['exact_match']['rate'], d['exact_match']['sample'], 'tok ms %.4f' % d['stage_ms_per_step']['tokenize'], 'frac %.4f' % d['roofline']['frac'])"
done
cat $out/host_path.json
