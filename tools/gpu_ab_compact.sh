#!/bin/bash
# A/B of the compaction kernels: flat U=8 default, flat with 16-byte stores (U = 1, 2, 4)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/ab_libs.sh dp-tokenization_amd/dptok/libdpt.so dp-tokenization_amd/csrc/build/var_v4u1/libdpt.so dp-tokenization_amd/csrc/build/var_v4u2/libdpt.so dp-tokenization_amd/csrc/build/var_v4u4/libdpt.so dp-tokenization_amd/dptok/libdpt.so > gpurun_out/ab.log 2>&1
rc=$?; cat gpurun_out/ab.log; exit $rc
