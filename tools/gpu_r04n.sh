#!/bin/bash
# round 4: the finish pass's shape (FIN_U loads in flight 8 / 16 / 32, FIN_THREADS 256 / 512 / 1024) on
# cfg2 1M and 125k, and the 64-lane kernel's waves per SIMD (5 / 6 / 7) on BLOOM after PUSH32;
# variant libraries built from the working tree with one constant changed; two interleaved rounds
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/r04n; mkdir -p $out
B=dp-tokenization_amd/csrc/build
for r in 1 2; do
  for v in head finu4 finu8 finu12 finu8t4k finu8t1k; do
    for args in "--workload cfg2" "--workload cfg2 --strings 125000"; do
      tag=${v}_$(echo $args | tr -d ' -')_$r
      lib=""; [ $v != head ] && lib="DPT_LIB=$PWD/$B/var_$v/libdpt.so"
      env $lib timeout -k 10 300 python bench.py $args --steps 20 --warmup 3 --no-cpu-baseline --exact-sample 65536 > $out/bench_$tag.log 2>&1 || { tail -5 $out/bench_$tag.log; exit 1; }
      tail -1 $out/bench_$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', 'GB/s %.2f' % (d['value']/1e9), 'ms %.4f' % d['ms_per_step'], 'exact', d['exact_match']['rate'], 'tok', round(d['stage_ms_per_step']['tokenize'],4))"
    done
  done
  for v in; do
    tag=${v}_bloom_$r
    lib=""; [ $v != head ] && lib="DPT_LIB=$PWD/$B/var_$v/libdpt.so"
    env $lib timeout -k 10 400 python bench.py --workload bloom --steps 10 --warmup 3 --no-cpu-baseline --exact-sample 65536 > $out/bench_$tag.log 2>&1 || { tail -5 $out/bench_$tag.log; exit 1; }
    tail -1 $out/bench_$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', 'GB/s %.2f' % (d['value']/1e9), 'ms %.4f' % d['ms_per_step'], 'exact', d['exact_match']['rate'], 'tok', round(d['stage_ms_per_step']['tokenize'],4))"
  done
done
