#!/bin/bash
# round 4: the slot-rounds wave count at every call size (var_sra with DPT_SR_ALL=1) against HEAD (the rule
# only below ~150k strings, else the occupancy limit), at 250k / 500k / 1M and cfg4, interleaved twice.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r04z2; mkdir -p $out
for r in 1 2; do
  for v in head sra; do
    lib=dp-tokenization_amd/dptok/libdpt.so; e=DPT_X=0
    [ $v = sra ] && { lib=dp-tokenization_amd/csrc/build/var_sra/libdpt.so; e=DPT_SR_ALL=1; }
    for wl in "250k --strings 250000 --steps 40 --warmup 5" "500k --strings 500000 --steps 40 --warmup 5" "1M --strings 1000000 --steps 20 --warmup 5" "cfg4 --workload cfg4 --steps 10 --warmup 3"; do
      set -- $wl; w=$1; shift
      tag=${v}_${w}_$r
      env $e DPT_LIB=$PWD/$lib timeout -k 10 300 python -u bench.py "$@" --no-cpu-baseline --exact-sample 65536 > $out/$tag.log 2>&1 || { tail -5 $out/$tag.log; exit 1; }
      tail -1 $out/$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', 'GB/s %.2f' % (d['value']/1e9), 'ms %.4f' % d['ms_per_step'], 'exact', d['exact_match']['rate'], 'tok %.4f' % d['stage_ms_per_step']['tokenize'])"
    done
  done
done
