#!/bin/bash
# Interleaved A/B of libdpt.so builds without the profiler: R repetitions of (every lib x every
# workload), bench.py's own HIP-event timing.  Usage: R=3 bash tools/gpu_ab_rep.sh <tag> lib1 lib2 ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/$1; shift; mkdir -p $out
for rep in $(seq 1 ${R:-3}); do
  for args in "--workload cfg2" "--workload cfg2 --strings 125000" "--workload cfg4" "--workload cfg5"; do
    for lib in "$@"; do
      tag=$(basename $(dirname $lib))
      wtag=$(echo $args | tr -d ' -')
      DPT_LIB=$PWD/$lib timeout -k 10 300 python3 bench.py $args --steps 20 --warmup 5 --no-cpu-baseline --exact-sample 16384 > $out/$tag.$wtag.$rep.log 2>&1 || { tail -5 $out/$tag.$wtag.$rep.log; exit 1; }
      grep '^{' $out/$tag.$wtag.$rep.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('%d %-10s %-34s GB/s %6.2f ms/step %.4f tokenize %.4f exact %s' % ($rep, '$tag', '$args', d['value']/1e9, d['ms_per_step'], d['stage_ms_per_step']['tokenize'], d['exact_match']['rate']))"
    done
  done
done
