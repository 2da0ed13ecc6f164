#!/bin/bash
# round 3: LANE_PF (lane-mode B reads the next position's candidates a step ahead) A/B on cfg4/cfg2/cfg5,
# the finish-pass fold A/B at 125k / 250k (var_nofold = no fold, no prefetch; var_lanepf0 = fold, no prefetch),
# kernel trace at 125k, BLOOM
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/round_r03y; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { tail -40 $out/pytest_gpu.log; exit 1; }
tail -1 $out/pytest_gpu.log
B=dp-tokenization_amd/csrc/build
H=dp-tokenization_amd/dptok/libdpt.so
for r in 1 2; do
  bash tools/ab_libs_wl.sh cfg4 $H $B/var_lanepf0/libdpt.so $B/var_lanepf1/libdpt.so || exit 1
done
bash tools/ab_libs_wl.sh cfg2 $H $B/var_lanepf0/libdpt.so $B/var_lanepf1/libdpt.so || exit 1
bash tools/ab_libs_wl.sh cfg5 $H $B/var_lanepf0/libdpt.so || exit 1
for r in 1 2; do
  for lib in $B/var_nofold/libdpt.so $B/var_lanepf0/libdpt.so $H; do
    for n in 125000 250000; do
      DPT_LIB=$PWD/$lib timeout -k 10 300 python -u bench.py --strings $n --steps 40 --warmup 5 --no-cpu-baseline --exact-sample 20000 > $out/s.log 2>&1 || { tail -20 $out/s.log; exit 1; }
      tail -1 $out/s.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$(basename $(dirname $lib))', $n, 'GB/s %.2f' % (d['value']/1e9), 'ms/step %.4f' % d['ms_per_step'], 'tok %.4f' % d['stage_ms_per_step']['tokenize'], 'exact', d['exact_match']['rate'])"
    done
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof125k -o run -- python3 bench.py --strings 125000 --steps 20 --warmup 3 --no-cpu-baseline > $out/trace125k.log 2>&1 || { tail -20 $out/trace125k.log; exit 1; }
find $out/prof125k -name "*kernel_stats.csv" -exec cut -c1-150 {} \;
bash tools/ab_libs_wl.sh bloom $H || exit 1
