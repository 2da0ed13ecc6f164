#!/bin/bash
# round 4: BLOOM's phase A walker -- 16-byte slots with the child filter (slot16) instead of the 8-byte
# ones, and the batched refill threshold A_REFILL64 16 / 48 (HEAD 32); two interleaved rounds
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/r04r; mkdir -p $out
B=dp-tokenization_amd/csrc/build
for r in 1 2; do
  for v in head slot16 ar64_16 ar64_48; do
    tag=${v}_bloom_$r
    lib=""; [ $v != head ] && lib="DPT_LIB=$PWD/$B/var_$v/libdpt.so"
    env $lib timeout -k 10 400 python bench.py --workload bloom --steps 10 --warmup 3 --no-cpu-baseline --exact-sample 65536 > $out/bench_$tag.log 2>&1 || { tail -5 $out/bench_$tag.log; exit 1; }
    tail -1 $out/bench_$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', 'GB/s %.2f' % (d['value']/1e9), 'ms %.4f' % d['ms_per_step'], 'exact', d['exact_match']['rate'], 'tok', round(d['stage_ms_per_step']['tokenize'],4))"
  done
done
