#!/bin/bash
# round 4: self-copy v2 (tagged counts, look-back publication, copy steps every few rounds), the merged
# fallback kernel and the interleaved LDS slots -- the full GPU suite, then an A/B against round 3's
# HEAD (var_r03) with the self-copy on / off on cfg2 1M, cfg2 125k and cfg4, and the per-call floor.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/r04c; mkdir -p $out
[ -z "$SKIP_SUITE" ] && { timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/pytest_gpu.txt 2>&1 || { tail -40 $out/pytest_gpu.txt; exit 1; }
tail -3 $out/pytest_gpu.txt
timeout -k 10 300 python tools/percall.py 2000 > $out/percall.json 2>&1 || { tail -5 $out/percall.json; exit 1; }
cat $out/percall.json; }
R03=dp-tokenization_amd/csrc/build/var_r03/libdpt.so
for r in 1 2; do
  for v in r03 sc0 sc1; do
    for args in "--workload cfg2" "--workload cfg2 --strings 125000" "--workload cfg4"; do
      tag=${v}_$(echo $args | tr -d ' -')_$r
      lib=""; sc=1
      [ $v = r03 ] && lib="DPT_LIB=$PWD/$R03"
      [ $v = sc0 ] && sc=0
      env $lib DPT_SELF_COPY=$sc timeout -k 10 300 python bench.py $args --steps 10 --warmup 3 --no-cpu-baseline --exact-sample 262144 > $out/bench_$tag.log 2>&1 || { tail -5 $out/bench_$tag.log; exit 1; }
      tail -1 $out/bench_$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); sc=d.get('self_copy') or {}; print('$tag', 'GB/s %.2f' % (d['value']/1e9), 'ms %.3f' % d['ms_per_step'], 'exact', d['exact_match']['rate'], 'sc', sc.get('strings_copied_by_first_pass'), 'tok', {k: round(v,3) for k,v in d['stage_ms_per_step'].items()})"
    done
  done
done
