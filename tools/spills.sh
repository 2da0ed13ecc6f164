#!/bin/bash
# Register/spill/occupancy summary of the tokenize kernels (compile only, no GPU): tools/spills.sh [-DKNOB=v ...]
cd "$(dirname "$0")/../dp-tokenization_amd/csrc"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -mllvm -amdgpu-sched-strategy=iterative-ilp "$@" \
  -c dpt_kernels.hip -o /tmp/spills_k.o -Rpass-analysis=kernel-resource-usage 2>&1 | python3 -c '
import re, sys
cur = None; rows = []
for ln in sys.stdin:
    m = re.search(r"Function Name: (\S+)", ln)
    if m: cur = {"name": m.group(1)}; rows.append(cur); continue
    m = re.search(r"remark: (?:\S+: )?\s*([A-Za-z ]+?)(?: \[bytes/lane\])?: (\d+)", ln)
    if m and cur is not None: cur[m.group(1).strip()] = m.group(2)
for r in rows:
    if "tokenize" not in r["name"] and "finish" not in r["name"]: continue
    n = re.sub(r"^_ZN3dpt\d+", "", r["name"]).replace("EEEvNS_8KernArgsE", "")
    print("%-48s vgpr %3s sgpr %3s spillS %3s spillV %3s scratch %3s occ %s LDS %s" % (n, r.get("VGPRs"), r.get("SGPRs"),
          r.get("SGPRs Spill"), r.get("VGPRs Spill"), r.get("ScratchSize"), r.get("Occupancy"), r.get("LDS Size")))
'
