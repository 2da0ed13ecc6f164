#!/bin/bash
# One GPU session for the strong-scaling evidence (SURVEY.md §8e, cfg3 = 1M strings split over
# the ranks): GPU parity suite, the default bench line, the 1-GPU points at the per-rank shard
# sizes of 2/4/8-way strong scaling (500k / 250k / 125k strings), and a 2-rank rehearsal of the
# strong path on the one card (gloo).  Every GPU step has its own time limit; stop at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/scale_${1:-r02}; mkdir -p $out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail -20 $out/smoke.log; exit 1; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { tail -30 $out/pytest_gpu.log; exit 1; }
tail -2 $out/pytest_gpu.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $out/bench_1m.log 2>&1 || { tail -20 $out/bench_1m.log; exit 1; }
tail -1 $out/bench_1m.log > $out/bench_1m.json
for n in 500000 250000 125000; do
  timeout -k 10 300 python -u bench.py --strings $n --steps 40 --warmup 5 --no-cpu-baseline > $out/bench_$n.log 2>&1 || { tail -20 $out/bench_$n.log; exit 1; }
  tail -1 $out/bench_$n.log > $out/bench_$n.json
done
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 \
    bench.py --gpus 2 --steps 10 --warmup 3 --no-cpu-baseline --dist-backend gloo > $out/rehearse_2rank.log 2>&1 || { tail -20 $out/rehearse_2rank.log; exit 1; }
grep '^{' $out/rehearse_2rank.log > $out/rehearse_2rank.json
for f in $out/bench_*.json $out/rehearse_2rank.json; do
  python3 -c "import json,sys; d=json.loads(open('$f').read()); print('$f', '%.2f GB/s' % (d['value']/1e9), 'ms/step %.3f' % d['ms_per_step'], 'exact', d['exact_match']['rate'], d['exact_match']['sample'], 'stages', d['stage_ms_per_step'], 'frac %.4f' % d['roofline']['frac'])"
done
