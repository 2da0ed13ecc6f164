#!/bin/bash
# A/B of libdpt.so variants (built with `make variant`) on cfg2: the bench line and the rocprof
# kernel stats of the tokenize and finish kernels.  Usage: bash tools/gpu_ab_tok.sh <tag> lib1 lib2 ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/$1; shift; mkdir -p $out
for lib in "$@"; do
  tag=$(basename $(dirname $lib))
  DPT_LIB=$PWD/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/$tag -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --exact-sample 65536 > $out/$tag.log 2>&1 || { tail -5 $out/$tag.log; exit 1; }
  grep '^{' $out/$tag.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', 'GB/s %.2f' % (d['value']/1e9), 'ms/step %.4f' % d['ms_per_step'], 'exact', d['exact_match']['rate'])"
  grep -E "tokenize_kernel<256|finish" $out/$tag/run_kernel_stats.csv | awk -F'",' '{split($2,a,","); printf "   %-60s avg_ms %.4f\n", substr($1,1,60), a[3]/1e6}'
done
