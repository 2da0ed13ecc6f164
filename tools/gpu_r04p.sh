#!/bin/bash
# round 4: s_memtime stamps by phase (libdpt_stamps.so, HEAD source) for BLOOM (100k strings, 64-lane
# kernel), cfg2 and cfg4 shapes -- where the 64-lane kernel's wave time goes
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/r04p; mkdir -p $out
timeout -k 10 600 python3 tools/prof_driver.py 100000 1 bloom gen-only > $out/gen.log 2>&1 || { tail -5 $out/gen.log; exit 1; }
timeout -k 10 300 python3 tools/prof_driver.py 200000 1 s2orc gen-only > $out/gen2.log 2>&1 || { tail -5 $out/gen2.log; exit 1; }
for a in "100000 256 bloom" "1000000 256 ascii" "200000 256 s2orc"; do
  timeout -k 10 300 python3 tools/stamps.py $a > $out/stamps_$(echo $a | tr ' ' _).txt 2>&1 || { tail -5 $out/stamps_$(echo $a | tr ' ' _).txt; exit 1; }
  grep -v amdgpu.ids $out/stamps_$(echo $a | tr ' ' _).txt
done
