#!/bin/bash
# A/B of libdpt.so builds over the workloads (cfg2 1M, cfg2 125k, cfg4, cfg5): the bench line and the
# tokenize kernel's rocprof average.  Usage: bash tools/gpu_ab_wl.sh <tag> lib1 lib2 ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/$1; shift; mkdir -p $out
for lib in "$@"; do
  tag=$(basename $(dirname $lib))
  for args in "--workload cfg2" "--workload cfg2 --strings 125000" "--workload cfg4" "--workload cfg5"; do
    wtag=$(echo $args | tr -d ' -')
    DPT_LIB=$PWD/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/$tag.$wtag -o run --output-format csv -- python3 bench.py $args --steps 10 --warmup 3 --no-cpu-baseline --exact-sample 65536 > $out/$tag.$wtag.log 2>&1 || { tail -5 $out/$tag.$wtag.log; exit 1; }
    tk=$(grep -E "tokenize_kernel<256" $out/$tag.$wtag/run_kernel_stats.csv | awk -F'",' '{split($2,a,","); printf "%.4f", a[3]/1e6}')
    grep '^{' $out/$tag.$wtag.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('%-10s %-28s GB/s %6.2f ms/step %.4f tokenize %s exact %s' % ('$tag', '$args', d['value']/1e9, d['ms_per_step'], '$tk', d['exact_match']['rate']))"
  done
done
