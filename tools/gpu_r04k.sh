#!/bin/bash
# round 4: per-call A/B on one box (DPT_NO_SOLO: the finish kernel back), twice, and per-phase stamps of
# a one-string call
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/r04k; mkdir -p $out
for r in 1 2; do
  for v in solo nosolo; do
    e=""; [ $v = nosolo ] && e="DPT_NO_SOLO=1"
    env $e timeout -k 10 300 python tools/percall.py 3000 > $out/percall_${v}_$r.json 2>/dev/null || { echo fail; exit 1; }
    echo $v $r; cat $out/percall_${v}_$r.json
  done
done
STAMP_REPS=500 timeout -k 10 120 python3 tools/stamps.py 1 > $out/stamps_1.txt 2>&1 && cat $out/stamps_1.txt
timeout -k 10 300 python tools/overlap_probe.py 10 > $out/overlap.json 2>&1; tail -2 $out/overlap.json
timeout -k 10 600 python -u -m pytest tests/test_gpu_pipeline.py -x -v --timeout 200 --timeout-method thread > $out/pytest_pipe.txt 2>&1 || { tail -40 $out/pytest_pipe.txt; exit 1; }
tail -3 $out/pytest_pipe.txt
for a in "--pipeline" ""; do
  for w in "--workload cfg2" "--workload cfg2 --strings 125000" "--workload cfg4"; do
    timeout -k 10 300 python bench.py $w $a --steps 10 --warmup 3 --no-cpu-baseline --exact-sample 65536 > $out/bench.log 2>&1 || { tail -5 $out/bench.log; exit 1; }
    tail -1 $out/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$w $a', 'GB/s %.2f' % (d['value']/1e9), 'ms %.3f' % d['ms_per_step'], 'exact', d['exact_match']['rate'], 'pipe', d['csr_pipeline'])"
  done
done
