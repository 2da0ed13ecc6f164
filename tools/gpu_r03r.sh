#!/bin/bash
# round 3: finish pass with quad copies (FIN_QUAD) -- GPU suite, then A/B vs id-per-thread copies
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r03r
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r03r/pytest.log 2>&1 || { tail -40 gpurun_out/r03r/pytest.log; exit 1; }
tail -1 gpurun_out/r03r/pytest.log
B=dp-tokenization_amd/csrc/build
for n in 125000 1000000; do
  for lib in dp-tokenization_amd/dptok/libdpt.so $B/var_fq0/libdpt.so; do
    DPT_LIB=$PWD/$lib timeout -k 10 300 python -u bench.py --strings $n --steps 40 --warmup 5 --no-cpu-baseline --exact-sample 65536 > gpurun_out/r03r/s.log 2>&1 || { tail -20 gpurun_out/r03r/s.log; exit 1; }
    tail -1 gpurun_out/r03r/s.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib'.split('/')[-2], $n, '%.2f GB/s' % (d['value']/1e9), 'ms/step %.4f' % d['ms_per_step'], 'tok %.4f' % d['stage_ms_per_step']['tokenize'], 'exact', d['exact_match']['rate'])"
  done
done
