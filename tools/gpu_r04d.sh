#!/bin/bash
# round 4: where the self-copy-off path lost time against round 3 -- one bench per library (git revisions
# built by tools/build_rev.sh; nosc = HEAD without the self-copy code, DPT_NO_SC), all with DPT_SELF_COPY=0
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/r04d; mkdir -p $out
B=dp-tokenization_amd/csrc/build
for r in 1 2; do
  for v in ${VARIANTS:-r03 prune hp merge nosc head}; do
    for args in "--workload cfg2" "--workload cfg2 --strings 125000" "--workload cfg4"; do
      tag=${v}_$(echo $args | tr -d ' -')_$r
      lib=""
      [ $v != head ] && lib="DPT_LIB=$PWD/$B/var_$v/libdpt.so"
      env $lib DPT_SELF_COPY=${SC:-0} timeout -k 10 300 python bench.py $args --steps 10 --warmup 3 --no-cpu-baseline --exact-sample 65536 > $out/bench_$tag.log 2>&1 || { tail -5 $out/bench_$tag.log; exit 1; }
      tail -1 $out/bench_$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); sc=d.get('self_copy') or {}; print('$tag', 'GB/s %.2f' % (d['value']/1e9), 'ms %.3f' % d['ms_per_step'], 'exact', d['exact_match']['rate'], 'sc', sc.get('strings_copied_by_first_pass'), 'tok', {k: round(v,3) for k,v in d['stage_ms_per_step'].items()})"
    done
  done
done
