#!/bin/bash
# round 3: batch-scan fold into the finish pass (fin_fold) + batched push edges in forward_lanes64:
# GPU suite, BLOOM A/B over PUSH_B, strong-scaling points
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/round_r03x; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { tail -40 $out/pytest_gpu.log; exit 1; }
tail -1 $out/pytest_gpu.log
B=dp-tokenization_amd/csrc/build
bash tools/ab_libs_wl.sh bloom dp-tokenization_amd/dptok/libdpt.so $B/var_pushb1/libdpt.so $B/var_pushb2/libdpt.so || exit 1
bash tools/ab_libs_wl.sh bloom dp-tokenization_amd/dptok/libdpt.so $B/var_pushb1/libdpt.so $B/var_pushb2/libdpt.so || exit 1
for n in 125000 250000 500000 1000000; do
  timeout -k 10 300 python -u bench.py --strings $n --steps 40 --warmup 5 --no-cpu-baseline > $out/strong_$n.log 2>&1 || { tail -20 $out/strong_$n.log; exit 1; }
  tail -1 $out/strong_$n.log > $out/strong_$n.json
  python3 -c "import json; d=json.load(open('$out/strong_$n.json')); print($n, 'GB/s %.2f' % (d['value']/1e9), 'ms/step %.4f' % d['ms_per_step'], 'tok %.4f' % d['stage_ms_per_step']['tokenize'], 'exact', d['exact_match']['rate'])"
done
