#!/bin/bash
# round 4: one-string host-path calls in one launch (EncodeLaunch::solo) -- the host-path and drop-in
# GPU tests, the per-call timings and a per-call kernel trace
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/r04j; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest.txt 2>&1 || { tail -40 $out/pytest.txt; exit 1; }
tail -2 $out/pytest.txt
timeout -k 10 300 python tools/percall.py 2000 > $out/percall.json 2>&1 && cat $out/percall.json
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $out/pc -o pc --output-format csv -- python3 tools/percall_trace.py 300 > $out/pc.log 2>&1 || { tail -5 $out/pc.log; exit 1; }
cut -c1-150 $out/pc/pc_kernel_stats.csv
