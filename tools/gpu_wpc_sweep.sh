#!/bin/bash
# Wave-count sweep (GPU box): the timeline build's split (tools/wave_timeline.py) and the product bench line at
# each forced resident-wave count.  Usage: bash tools/gpu_wpc_sweep.sh <tag> <strings> <w1> <w2> ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=$1; n=$2; shift 2; out=gpurun_out/$tag; mkdir -p $out
for w in "$@"; do
  DPT_NO_SMALL_WPC=1 DPT_WAVES_PER_CU=$w timeout -k 10 200 python -u tools/wave_timeline.py ascii $n > $out/wt_${n}_w$w.log 2>&1 || { tail -5 $out/wt_${n}_w$w.log; exit 1; }
  DPT_NO_SMALL_WPC=1 DPT_WAVES_PER_CU=$w timeout -k 10 200 python -u bench.py --strings $n --steps 40 --warmup 5 --no-cpu-baseline > $out/b_${n}_w$w.log 2>&1 || { tail -5 $out/b_${n}_w$w.log; exit 1; }
  python3 - $out/wt_${n}_w$w.log $out/b_${n}_w$w.log $w <<'PY'
import json, sys
t = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")][-1]
b = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print("w=%s span %.1f tail %.1f ramp %.1f rounds %.2f round %.1f | bench %.2f GB/s tok %.4f ms step %.4f" % (
    sys.argv[3], t["span_us"], t["tail_us"], t["ramp_us"], t["rounds_per_wave"], t["round_us_by_busy"]["4"][1],
    b["value"] / 1e9, b["stage_ms_per_step"]["tokenize"], b["ms_per_step"]))
PY
done
