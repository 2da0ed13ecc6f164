#!/bin/bash
# round 4: the small-call waves rule at ~6 instead of ~7 strings per slot (125k: 21 instead of 18 waves
# per CU), at 100k / 125k / 150k strings, interleaved twice.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r04x2; mkdir -p $out
for r in 1 2; do
  for lib in dp-tokenization_amd/dptok/libdpt.so dp-tokenization_amd/csrc/build/var_spr6/libdpt.so; do
    for n in 100000 125000 150000; do
      tag=$(basename $(dirname $lib))_${n}_$r
      DPT_LIB=$PWD/$lib timeout -k 10 300 python -u bench.py --strings $n --steps 40 --warmup 5 --no-cpu-baseline --exact-sample 65536 > $out/$tag.log 2>&1 || { tail -5 $out/$tag.log; exit 1; }
      tail -1 $out/$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', 'GB/s %.2f' % (d['value']/1e9), 'ms %.4f' % d['ms_per_step'], 'exact', d['exact_match']['rate'], 'tok %.4f' % d['stage_ms_per_step']['tokenize'])"
    done
  done
done
