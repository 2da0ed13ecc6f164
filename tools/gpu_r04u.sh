#!/bin/bash
# round 4: the finish pass's grid target (FIN_TARGET_BLOCKS; only calls under 2048 batches split a batch
# over slices, so 1M never saw it) at the strong-scaling shard sizes -- 2048 (HEAD) vs 512 / 1024 / 4096,
# interleaved twice.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r04u; mkdir -p $out
B=dp-tokenization_amd/csrc/build
for r in 1 2; do
  for lib in dp-tokenization_amd/dptok/libdpt.so $B/var_ftb512/libdpt.so $B/var_ftb1024/libdpt.so $B/var_ftb4096/libdpt.so; do
    for n in 125000 250000 500000; do
      tag=$(basename $(dirname $lib))_${n}_$r
      DPT_LIB=$PWD/$lib timeout -k 10 300 python -u bench.py --strings $n --steps 40 --warmup 5 --no-cpu-baseline --exact-sample 65536 > $out/$tag.log 2>&1 || { tail -5 $out/$tag.log; exit 1; }
      tail -1 $out/$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', 'GB/s %.2f' % (d['value']/1e9), 'ms %.4f' % d['ms_per_step'], 'exact', d['exact_match']['rate'], 'tok %.4f' % d['stage_ms_per_step']['tokenize'])"
    done
  done
done
