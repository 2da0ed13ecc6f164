#!/bin/bash
# rocprofv3 kernel stats of the histogram kernel for alternative builds (DPT_LIB=path each)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for lib in "$@"; do
  tag=$(basename $(dirname $lib))
  DPT_LIB=$PWD/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/hist_$tag -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --exact-sample 1000 > gpurun_out/hist_$tag.log 2>&1 || exit 1
  echo "$tag $(grep -h hist_kernel $(find gpurun_out/hist_$tag -name '*kernel_stats.csv') | cut -d, -f4)"
done
