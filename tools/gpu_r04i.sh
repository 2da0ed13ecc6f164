#!/bin/bash
# round 4: the full GPU suite at HEAD (self-copy compiled out of the product library; its tests also run
# on build/var_sc) and the default bench line
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/r04i; mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/pytest_gpu.txt 2>&1 || { tail -40 $out/pytest_gpu.txt; exit 1; }
tail -3 $out/pytest_gpu.txt
timeout -k 10 300 python bench.py > $out/bench.json 2> $out/bench.err || { tail -5 $out/bench.err; exit 1; }
cut -c1-400 $out/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $out/pc -o pc --output-format csv -- python3 tools/percall_trace.py 300 > $out/pc.log 2>&1 || { tail -5 $out/pc.log; exit 1; }
timeout -k 10 300 python tools/percall.py 2000 > $out/percall.json 2>&1 && cat $out/percall.json
