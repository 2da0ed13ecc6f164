#!/bin/bash
# round 4: one-string calls on the 64-lane kernel -- host-path tests, then per-call A/B on one box:
# solo (64-lane), solo16 (DPT_SOLO16: the 16-lane row), nosolo (DPT_NO_SOLO: the four-step chain), twice
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/r04m; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_hostpath.py tests/test_compat.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > $out/pytest.txt 2>&1 || { tail -30 $out/pytest.txt; exit 1; }
tail -2 $out/pytest.txt
for r in 1 2; do
  for v in solo solo16 nosolo; do
    e=""; [ $v = nosolo ] && e="DPT_NO_SOLO=1"; [ $v = solo16 ] && e="DPT_SOLO16=1"
    env $e timeout -k 10 300 python tools/percall.py 3000 > $out/percall_${v}_$r.json 2>/dev/null || { echo fail; exit 1; }
    echo $v $r $(python3 -c "import json; d=json.load(open('$out/percall_${v}_$r.json')); print({k: round(d[k],1) for k in ('dp_tokenize_us','encode_csr_us','dpt_encode_device_sync_us')})")
  done
done
