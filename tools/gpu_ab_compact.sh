#!/bin/bash
# A/B of the compaction kernels on cfg2 and cfg5: the flat kernel (default) and the per-string
# kernel (DPT_COMPACT_OLD=1); stage times in each line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=dp-tokenization_amd/dptok/libdpt.so
for wl in cfg2 cfg5; do
  bash tools/ab_libs_wl.sh $wl $L || exit 1
  DPT_COMPACT_OLD=1 bash tools/ab_libs_wl.sh $wl $L | sed 's/^/old: /' || exit 1
done
