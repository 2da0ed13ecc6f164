#!/bin/bash
# Finish-kernel A/B at two batch sizes (1M and 125k cfg2 strings): rocprof avg of the finish and
# tokenize kernels and the bench line.  Usage: bash tools/gpu_ab_fin.sh <tag> lib1 lib2 ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/$1; shift; mkdir -p $out
for lib in "$@"; do
  tag=$(basename $(dirname $lib))
  for n in 1000000 125000; do
    DPT_LIB=$PWD/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/$tag.$n -o run --output-format csv -- python3 bench.py --strings $n --steps 20 --warmup 3 --no-cpu-baseline --exact-sample 65536 > $out/$tag.$n.log 2>&1 || { tail -5 $out/$tag.$n.log; exit 1; }
    grep '^{' $out/$tag.$n.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', $n, 'GB/s %.2f' % (d['value']/1e9), 'ms/step %.4f' % d['ms_per_step'], 'exact', d['exact_match']['rate'])"
    grep -E "tokenize_kernel<256|finish" $out/$tag.$n/run_kernel_stats.csv | awk -F'",' '{split($2,a,","); printf "   %-50s avg_ms %.4f\n", substr($1,1,50), a[3]/1e6}'
  done
done
