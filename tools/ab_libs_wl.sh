#!/bin/bash
# A/B alternative builds of libdpt.so on one workload: bash tools/ab_libs_wl.sh <cfg2|cfg4|cfg5> lib...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
wl=$1; shift
for lib in "$@"; do
  tag=$(basename $(dirname $lib))_$wl; [ "$tag" = "dptok_$wl" ] && tag=head_$wl
  DPT_LIB=$PWD/$lib timeout -k 10 300 python bench.py --workload $wl --steps 10 --warmup 3 --no-cpu-baseline --exact-sample 65536 > gpurun_out/bench_$tag.log 2>&1 || { tail -5 gpurun_out/bench_$tag.log; exit 1; }
  tail -1 gpurun_out/bench_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', 'GB/s %.2f' % (d['value']/1e9), 'exact', d['exact_match']['rate'], 'stages', {k: round(v,3) for k,v in d['stage_ms_per_step'].items()})"
done
