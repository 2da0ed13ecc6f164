#!/bin/bash
# Round-2 evidence session at HEAD: GPU suite, smoke, HBM traffic of the tokenize kernel
# (profiles/pmc_traffic.json), PMC summary, the headline line with the CPU baseline, its rocprof
# kernel stats, the strong-scaling 1-GPU points, cfg4 / cfg5 / bloom lines and the host-path line.
# Usage: bash tools/gpu_r02e.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=$1; out=gpurun_out/$tag; mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { tail -40 $out/pytest_gpu.log; exit 1; }
tail -1 $out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail -20 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 600 python3 tools/pmc_traffic.py 1000000 $tag > $out/traffic.log 2>&1 || { tail -20 $out/traffic.log; exit 1; }
cp gpurun_out/pmc_$tag/pmc_traffic.json $out/pmc_traffic.json
tail -1 $out/traffic.log
bash tools/pmc.sh $tag > $out/pmc.log 2>&1 || { tail -20 $out/pmc.log; exit 1; }
cp gpurun_out/pmc_$tag/summary.txt $out/pmc_summary.txt
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $out/bench.log 2>&1 || { tail -20 $out/bench.log; exit 1; }
tail -1 $out/bench.log > $out/bench.json; cat $out/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 10 --warmup 3 > $out/trace.log 2>&1 || { tail -20 $out/trace.log; exit 1; }
cut -c1-150 $out/trace/run_kernel_stats.csv | head -9
for n in 500000 250000 125000; do
  timeout -k 10 300 python -u bench.py --strings $n --steps 40 --warmup 5 --no-cpu-baseline > $out/bench_$n.log 2>&1 || { tail -20 $out/bench_$n.log; exit 1; }
  tail -1 $out/bench_$n.log > $out/bench_$n.json
done
for w in cfg4 cfg5; do
  timeout -k 10 400 python -u bench.py --workload $w --steps 10 --warmup 3 --no-cpu-baseline > $out/bench_$w.log 2>&1 || { tail -20 $out/bench_$w.log; exit 1; }
  tail -1 $out/bench_$w.log > $out/bench_$w.json
done
timeout -k 10 500 python -u bench.py --workload bloom --steps 10 --warmup 3 --no-cpu-baseline --exact-sample 100000 > $out/bench_bloom.log 2>&1 || { tail -20 $out/bench_bloom.log; exit 1; }
tail -1 $out/bench_bloom.log > $out/bench_bloom.json
timeout -k 10 300 python -u bench.py --host-path > $out/host.log 2>&1 || { tail -20 $out/host.log; exit 1; }
tail -1 $out/host.log > $out/host_path.json
for f in $out/bench_*.json; do
  python3 -c "import json; d=json.loads(open('$f').read()); print('$f', '%.2f GB/s' % (d['value']/1e9), 'ms/step %.4f' % d['ms_per_step'], 'exact', d['exact_match']['rate'], d['exact_match']['sample'], 'tok ms %.4f' % d['stage_ms_per_step']['tokenize'], 'frac %.4f' % d['roofline']['frac'])"
done
