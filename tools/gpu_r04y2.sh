#!/bin/bash
# round 4: the small-call waves rule as the fewest slot-rounds (w * ceil(rounds), smallest w on ties)
# against the previous ~7-strings-per-slot rule (var_head) at 50k / 75k / 100k / 125k strings,
# interleaved twice (125k picks 18 waves per CU either way: a control).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r04y2; mkdir -p $out
for r in 1 2; do
  for lib in dp-tokenization_amd/csrc/build/var_head/libdpt.so dp-tokenization_amd/dptok/libdpt.so; do
    for n in 50000 75000 100000 125000; do
      tag=$(basename $(dirname $lib))_${n}_$r
      DPT_LIB=$PWD/$lib timeout -k 10 300 python -u bench.py --strings $n --steps 40 --warmup 5 --no-cpu-baseline --exact-sample 65536 > $out/$tag.log 2>&1 || { tail -5 $out/$tag.log; exit 1; }
      tail -1 $out/$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', 'GB/s %.2f' % (d['value']/1e9), 'ms %.4f' % d['ms_per_step'], 'exact', d['exact_match']['rate'], 'tok %.4f' % d['stage_ms_per_step']['tokenize'])"
    done
  done
done
