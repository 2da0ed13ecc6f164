#!/bin/bash
# round 4: first GPU run of the self-copy build -- its GPU tests (and the fold / sharded ones), then an
# A/B of the self-copy on / off (DPT_SELF_COPY, same library) on cfg2 1M, cfg2 125k and cfg4, then the
# r04a diagnostics (per-phase PMC, BLOOM profile, PUSH32 A/B) on the build without the self-copy code.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/r04b; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_selfcopy.py tests/test_gpu_fold.py tests/test_gpu_hostpath.py -x -v -s --timeout 200 --timeout-method thread > $out/pytest_sc.txt 2>&1 || { tail -40 $out/pytest_sc.txt; exit 1; }
tail -3 $out/pytest_sc.txt
timeout -k 10 300 python tools/percall.py 2000 > $out/percall.json 2>&1 || { tail -5 $out/percall.json; exit 1; }
cat $out/percall.json
for r in 1 2; do
  for sc in 0 1; do
    for args in "--workload cfg2" "--workload cfg2 --strings 125000" "--workload cfg4"; do
      tag=sc${sc}_$(echo $args | tr -d ' -')_$r
      DPT_SELF_COPY=$sc timeout -k 10 300 python bench.py $args --steps 10 --warmup 3 --no-cpu-baseline > $out/bench_$tag.log 2>&1 || { tail -5 $out/bench_$tag.log; exit 1; }
      tail -1 $out/bench_$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', 'GB/s %.2f' % (d['value']/1e9), 'ms %.3f' % d['ms_per_step'], 'exact', d['exact_match']['rate'], d.get('self_copy'), 'stages', {k: round(v,3) for k,v in d['stage_ms_per_step'].items()})"
    done
  done
done
