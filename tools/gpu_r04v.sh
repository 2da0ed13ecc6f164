#!/bin/bash
# round 4: exact rounds for the persistent grid (as few waves as run the same number of rounds) -- the
# same library with DPT_NO_EXACT_ROUNDS=1 (the previous grid) vs without, at the strong-scaling shard
# sizes, 1M, cfg4 and BLOOM, interleaved twice.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r04v; mkdir -p $out
run() {   # tag, env, bench args
  local tag=$1 envv=$2; shift 2
  env $envv timeout -k 10 300 python -u bench.py "$@" --no-cpu-baseline > $out/$tag.log 2>&1 || { tail -5 $out/$tag.log; return 1; }
  tail -1 $out/$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', 'GB/s %.2f' % (d['value']/1e9), 'ms %.4f' % d['ms_per_step'], 'exact', d['exact_match']['rate'], 'tok %.4f' % d['stage_ms_per_step']['tokenize'])"
}
for r in 1 2; do
  for v in old new; do
    e=DPT_NO_EXACT_ROUNDS=1; [ $v = new ] && e=DPT_X=0
    for n in 125000 250000 500000 1000000; do
      run ${v}_${n}_$r $e --strings $n --steps 40 --warmup 5 --exact-sample 65536 || exit 1
    done
    run ${v}_cfg4_$r $e --workload cfg4 --steps 10 --warmup 3 --exact-sample 65536 || exit 1
    run ${v}_bloom_$r $e --workload bloom --steps 10 --warmup 3 --exact-sample 65536 || exit 1
  done
done
