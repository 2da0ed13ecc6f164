#!/bin/bash
# round 3: FALLBACK_DIV 16 / 64 (smaller grids for the two usually-empty fallback passes; head = 4) at the strong-scaling sizes
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
B=dp-tokenization_amd/csrc/build
H=dp-tokenization_amd/dptok/libdpt.so
for r in 1 2 3; do
  for lib in $H $B/var_fbdiv16/libdpt.so $B/var_fbdiv64/libdpt.so; do
    for n in 125000 250000; do
      DPT_LIB=$PWD/$lib timeout -k 10 300 python -u bench.py --strings $n --steps 60 --warmup 5 --no-cpu-baseline --exact-sample 20000 > gpurun_out/s.log 2>&1 || { tail -20 gpurun_out/s.log; exit 1; }
      tail -1 gpurun_out/s.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$(basename $(dirname $lib))', $n, 'GB/s %.2f' % (d['value']/1e9), 'ms/step %.4f' % d['ms_per_step'], 'tok %.4f' % d['stage_ms_per_step']['tokenize'], 'exact', d['exact_match']['rate'])"
    done
  done
done
bash tools/ab_libs_wl.sh cfg4 $H $B/var_fbdiv64/libdpt.so || exit 1
