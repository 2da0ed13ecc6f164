#!/bin/bash
# round 3: lane-mode B for the 64-lane kernel (forward_lanes64): GPU suite, then BLOOM A/B against LANES64=0
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/round_r03v; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { tail -40 $out/pytest_gpu.log; exit 1; }
tail -1 $out/pytest_gpu.log
B=dp-tokenization_amd/csrc/build
bash tools/ab_libs_wl.sh bloom dp-tokenization_amd/dptok/libdpt.so $B/var_l64off/libdpt.so || exit 1
bash tools/ab_libs_wl.sh bloom dp-tokenization_amd/dptok/libdpt.so $B/var_l64off/libdpt.so || exit 1
timeout -k 10 400 python -u bench.py --workload bloom --steps 10 --warmup 3 > $out/bench_bloom.log 2>&1 || { tail -20 $out/bench_bloom.log; exit 1; }
tail -1 $out/bench_bloom.log > $out/bench_bloom.json
