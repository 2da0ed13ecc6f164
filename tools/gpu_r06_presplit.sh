#!/bin/bash
# Round 6 (GPU box): the new GPU tests (counter bias, llama-mode scale), then cfg2p / cfg4p bench lines and a
# kernel trace of cfg2p.  Usage: bash tools/gpu_r06_presplit.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=$1; out=gpurun_out/$tag; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py::test_long_pass_offsets_past_2g tests/test_gpu_scale_exact.py::test_presplit_llama_mode_prefix_exact -x -v --timeout 300 --timeout-method thread > $out/pytest_new.log 2>&1 || { tail -40 $out/pytest_new.log; exit 1; }
tail -3 $out/pytest_new.log
bash tools/gpu_quick.sh $tag cfg2 cfg2p cfg4 cfg4p || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace_cfg2p -o run --output-format csv -- python3 bench.py --workload cfg2p --no-cpu-baseline --steps 10 --warmup 3 --exact-sample 1000 > $out/trace_cfg2p.log 2>&1 || { tail -20 $out/trace_cfg2p.log; exit 1; }
find $out/trace_cfg2p -name "*kernel_stats.csv" | head -1 | xargs cat | cut -c1-160 | head -6
