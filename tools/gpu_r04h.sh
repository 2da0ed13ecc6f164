#!/bin/bash
# round 4: the product build (self-copy code compiled in, off by default) against the same source
# without it (var_nosc2, DPT_NO_SC): does the cold code's register cost show?  cfg2 1M / 125k / 250k,
# cfg4, bloom; two interleaved rounds
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/r04h; mkdir -p $out
B=dp-tokenization_amd/csrc/build
for r in 1 2; do
  for v in head nosc2; do
    for args in "--workload cfg2" "--workload cfg2 --strings 125000" "--workload cfg2 --strings 250000" "--workload cfg4" "--workload bloom"; do
      tag=${v}_$(echo $args | tr -d ' -')_$r
      lib=""
      [ $v != head ] && lib="DPT_LIB=$PWD/$B/var_$v/libdpt.so"
      env $lib timeout -k 10 300 python bench.py $args --steps 10 --warmup 3 --no-cpu-baseline --exact-sample 65536 > $out/bench_$tag.log 2>&1 || { tail -5 $out/bench_$tag.log; exit 1; }
      tail -1 $out/bench_$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', 'GB/s %.2f' % (d['value']/1e9), 'ms %.3f' % d['ms_per_step'], 'exact', d['exact_match']['rate'], 'tok', {k: round(v,3) for k,v in d['stage_ms_per_step'].items()})"
    done
  done
done
