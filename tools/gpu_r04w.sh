#!/bin/bash
# round 4: first-pass work partitions NPART 16 (HEAD) vs 8 / 32 (round 2 measured 32 equal under the single
# counter's design; the batch lines and interleaved partitions changed the claim pattern since), at 125k,
# 1M and cfg4, interleaved twice.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r04w; mkdir -p $out
B=dp-tokenization_amd/csrc/build
for r in 1 2; do
  for lib in dp-tokenization_amd/dptok/libdpt.so $B/var_np8/libdpt.so $B/var_np32/libdpt.so; do
    for wl in "125000 --strings 125000 --steps 40 --warmup 5" "1M --strings 1000000 --steps 20 --warmup 5" "cfg4 --workload cfg4 --steps 10 --warmup 3"; do
      set -- $wl; w=$1; shift
      tag=$(basename $(dirname $lib))_${w}_$r
      DPT_LIB=$PWD/$lib timeout -k 10 300 python -u bench.py "$@" --no-cpu-baseline --exact-sample 65536 > $out/$tag.log 2>&1 || { tail -5 $out/$tag.log; exit 1; }
      tail -1 $out/$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', 'GB/s %.2f' % (d['value']/1e9), 'ms %.4f' % d['ms_per_step'], 'exact', d['exact_match']['rate'], 'tok %.4f' % d['stage_ms_per_step']['tokenize'])"
    done
  done
done
