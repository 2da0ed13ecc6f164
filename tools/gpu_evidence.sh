#!/bin/bash
# Final evidence of a round (GPU box): GPU suite, smoke, HBM traffic (calibrated PMC passes -- BEFORE the
# bench, so its line reports the traffic of the same source), the default bench line (CPU baseline
# included), its rocprofv3 kernel trace + stats, the PMC summary; then the other workloads, the
# strong-scaling points, the host path and the per-call floor.
# Usage: bash tools/gpu_evidence.sh <tag> [1|2|2a|2b]   (part 1: up to the PMC summary; part 2: the rest = 2a (the other
# workloads and the strong-scaling points) + 2b (host path, per-call floor, cfg4p / BLOOM traces and PMC summaries))
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=$1; part=${2:-all}; out=gpurun_out/round_$tag; mkdir -p $out
if [ $part = 1 ] || [ $part = all ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { tail -40 $out/pytest_gpu.log; exit 1; }
tail -1 $out/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail -20 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 600 python3 tools/pmc_traffic.py 1000000 $tag > $out/traffic.log 2>&1 || { tail -20 $out/traffic.log; exit 1; }
tail -1 $out/traffic.log | cut -c1-300
timeout -k 10 400 python -u bench.py > $out/bench.log 2>&1 || { tail -20 $out/bench.log; exit 1; }
tail -1 $out/bench.log > $out/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 10 --warmup 3 > $out/trace.log 2>&1 || { tail -20 $out/trace.log; exit 1; }
bash tools/pmc.sh $tag > $out/pmc.log 2>&1 || { tail -20 $out/pmc.log; exit 1; }
cp gpurun_out/pmc_$tag/summary.txt $out/pmc_summary.txt 2>/dev/null
fi
[ $part = 1 ] && exit 0
if [ $part != 2b ]; then
for wl in cfg1 cfg4 cfg5 bloom cfg2p cfg4p; do
  timeout -k 10 400 python -u bench.py --workload $wl --steps 10 --warmup 3 > $out/bench_$wl.log 2>&1 || { tail -20 $out/bench_$wl.log; exit 1; }
  tail -1 $out/bench_$wl.log > $out/bench_$wl.json
done
for n in 500000 250000 125000; do
  timeout -k 10 300 python -u bench.py --strings $n --steps 40 --warmup 5 --no-cpu-baseline > $out/strong_$n.log 2>&1 || { tail -20 $out/strong_$n.log; exit 1; }
  grep '^{' $out/strong_$n.log | tail -1 > $out/strong_$n.json
done
for n in 500000 250000 125000; do   # the same shards with the per-step RCCL all-reduce the N > 1 runs do (world 1)
  DPT_BENCH_COLL=1 timeout -k 10 300 python -u bench.py --strings $n --steps 40 --warmup 5 --no-cpu-baseline > $out/strongc_$n.log 2>&1 || { tail -20 $out/strongc_$n.log; exit 1; }
  grep '^{' $out/strongc_$n.log | tail -1 > $out/strong_${n}_rccl.json
done
for n in 250000 125000; do   # the same shards with one batch in flight (bench.py --inflight 1)
  timeout -k 10 300 python -u bench.py --strings $n --steps 40 --warmup 5 --no-cpu-baseline --inflight 1 > $out/strong1_$n.log 2>&1 || { tail -20 $out/strong1_$n.log; exit 1; }
  grep '^{' $out/strong1_$n.log | tail -1 > $out/strong_${n}_inflight1.json
done
fi
[ $part = 2a ] && exit 0
for r in 1 2 3; do   # (three runs in one lease: the drop-in's spread across runs)
  timeout -k 10 400 python -u bench.py --host-path > $out/host_$r.log 2>&1 || { tail -20 $out/host_$r.log; exit 1; }
  tail -1 $out/host_$r.log > $out/host_path_$r.json
done
timeout -k 10 300 python tools/percall.py 3000 > $out/percall.json 2>/dev/null || { echo percall failed; exit 1; }
# llama mode (PRESPLIT, cfg4p): kernel trace + PMC summary of its first pass
bash tools/pmc.sh ${tag}_cfg4p 200000 s2orcp > $out/pmc_cfg4p.log 2>&1 || { tail -20 $out/pmc_cfg4p.log; exit 1; }
cp gpurun_out/pmc_${tag}_cfg4p/summary.txt $out/pmc_cfg4p_summary.txt 2>/dev/null
find gpurun_out/pmc_${tag}_cfg4p/trace -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $out/cfg4p_kernel_stats.csv
# BLOOM scale (the 64-lane ATOMS kernel): kernel trace + PMC summary
bash tools/pmc.sh ${tag}_bloom 500000 bloom > $out/pmc_bloom.log 2>&1 || { tail -20 $out/pmc_bloom.log; exit 1; }
cp gpurun_out/pmc_${tag}_bloom/summary.txt $out/pmc_bloom_summary.txt 2>/dev/null
find gpurun_out/pmc_${tag}_bloom/trace -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $out/bloom_kernel_stats.csv
for f in $(ls $out/bench.json $out/bench_*.json $out/strong_*.json 2>/dev/null); do
  python3 -c "import json; d=json.loads(open('$f').read()); print('$f', '%.2f GB/s' % (d['value']/1e9), 'ms/step %.4f' % d['ms_per_step'], 'exact', d['exact_match']['rate'], d['exact_match']['sample'], 'tok ms %.4f' % d['stage_ms_per_step']['tokenize'], 'frac %.4f' % d['roofline']['frac'], 'traffic', d['roofline'].get('traffic'))"
done
cat $out/percall.json
[ -d $out/trace ] && find $out/trace -name "*kernel_stats.csv" | head -1 | xargs cat | cut -c1-150 | head -8 || true
