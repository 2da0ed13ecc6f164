#!/bin/bash
# round 4: the pipelined calls' kernel trace (does the CSR pass overlap the next step's first pass, and
# what does it cost) and the LDS-free CSR pass alone in ordinary calls (DPT_LITE=1), cfg2 1M
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/r04o; mkdir -p $out
timeout -k 10 300 rocprofv3 --kernel-trace -d $out/pipe -o pipe --output-format csv -- python3 bench.py --pipeline --steps 6 --warmup 2 --no-cpu-baseline --exact-sample 4096 > $out/pipe.log 2>&1 || { tail -5 $out/pipe.log; exit 1; }
tail -1 $out/pipe.log | cut -c1-200
DPT_LITE=1 timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --exact-sample 65536 > $out/lite.log 2>&1 || { tail -5 $out/lite.log; exit 1; }
tail -1 $out/lite.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('lite (ordinary calls)', 'GB/s %.2f' % (d['value']/1e9), 'ms %.4f' % d['ms_per_step'], 'exact', d['exact_match']['rate'])"
