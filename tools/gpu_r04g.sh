#!/bin/bash
# round 4: self-copy v3 (batch lines, one-load look-back prefixes, offsets by the finish pass) -- its GPU
# tests, then cfg2 1M / 125k / cfg4 with the self-copy on and off, then per-phase stamps at 125k
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/r04g; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_selfcopy.py tests/test_gpu_fold.py tests/test_gpu_hostpath.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $out/pytest.txt 2>&1 || { tail -30 $out/pytest.txt; exit 1; }
tail -2 $out/pytest.txt
for sc in 1 0; do
  for args in "--workload cfg2" "--workload cfg2 --strings 125000" "--workload cfg4"; do
    tag=sc${sc}_$(echo $args | tr -d ' -')
    DPT_SELF_COPY=$sc timeout -k 10 300 python bench.py $args --steps 10 --warmup 3 --no-cpu-baseline --exact-sample 262144 > $out/bench_$tag.log 2>&1 || { tail -5 $out/bench_$tag.log; exit 1; }
    tail -1 $out/bench_$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); sc=d.get('self_copy') or {}; print('$tag', 'GB/s %.2f' % (d['value']/1e9), 'ms %.3f' % d['ms_per_step'], 'exact', d['exact_match']['rate'], 'sc', sc.get('strings_copied_by_first_pass'), sc.get('batches_copied_whole'), 'tok', {k: round(v,3) for k,v in d['stage_ms_per_step'].items()})"
  done
done
DPT_SELF_COPY=1 timeout -k 10 120 python3 tools/stamps.py 125000 > $out/stamps_sc1.txt 2>&1 && cat $out/stamps_sc1.txt
