#!/bin/bash
# round 4: fallback_kernel's early exit (both lists empty: no tickets, no waits) -- A/B against the
# previous HEAD's library at the 125k strong point and at 1M, interleaved twice; the kernel trace of the
# 125k point; then the GPU suite.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/r04t; mkdir -p $out
H=dp-tokenization_amd/csrc/build/var_head/libdpt.so
N=dp-tokenization_amd/dptok/libdpt.so
for r in 1 2; do
  for lib in $H $N; do
    for n in 125000 1000000; do
      tag=$(basename $(dirname $lib))_${n}_$r
      DPT_LIB=$PWD/$lib timeout -k 10 300 python -u bench.py --strings $n --steps 40 --warmup 5 --no-cpu-baseline > $out/$tag.log 2>&1 || { tail -5 $out/$tag.log; exit 1; }
      tail -1 $out/$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', 'GB/s %.2f' % (d['value']/1e9), 'ms %.4f' % d['ms_per_step'], 'exact', d['exact_match']['rate'], 'tok %.4f' % d['stage_ms_per_step']['tokenize'])"
    done
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace -o run --output-format csv -- python3 bench.py --strings 125000 --steps 20 --warmup 3 --no-cpu-baseline > $out/trace.log 2>&1 || { tail -5 $out/trace.log; exit 1; }
find $out/trace -name "*kernel_stats.csv" | head -1 | xargs cut -c1-140
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { tail -30 $out/pytest_gpu.log; exit 1; }
tail -1 $out/pytest_gpu.log
