"""Phase table from a tools/gpu_r04l.sh (or gpu_phase_wl.sh) log: per stop build, the tokenize kernel's
time and counters, and per phase (the increment between consecutive builds) the time, instructions, LDS
bank-conflict cycles against active LDS cycles (SQ_LDS_BANK_CONFLICT / SQ_ACTIVE_INST_LDS) and waits.
Usage: python tools/phase_table.py <log> [workload-suffix]"""
import re
import sys

names = {"var_stop1": "prep", "var_stop21": "+A0", "var_stop2": "+A walkers", "var_stop25": "+B cut points",
         "var_stop26": "+B chunk recurrence", "var_stop27": "+B transfer + fix-up", "var_stop3": "+C1 (lane walks)",
         "var_c2s1": "+C2 bulk", "var_c2s2": "+C2 hash", "dptok": "+C2 rest (full kernel)"}
order = ["var_stop1", "var_stop21", "var_stop2", "var_stop25", "var_stop26", "var_stop27", "var_stop3", "var_c2s1", "var_c2s2",
         "dptok"]
suffix = sys.argv[2] if len(sys.argv) > 2 else None
rows, cur, kern = {}, None, False
for line in open(sys.argv[1]):
    m = re.match(r"== (\S+)", line)
    if m:
        tag = m.group(1)
        base, _, wl = tag.rpartition("_")
        cur = None
        if suffix is None:   # (gpu_phase_wl.sh logs: the tag is the build's directory)
            cur = rows.setdefault(tag, {})
        elif wl == suffix:
            cur = rows.setdefault(base, {})
        kern = False
        continue
    if cur is None:
        continue
    if "tokenize_kernel<256" in line:
        kern = True
        try:
            cur["ns"] = float(line.split("avg_ns=")[1])
        except (IndexError, ValueError):
            pass
        continue
    if "tokenize_kernel<2048" in line or "finish" in line:
        kern = False
        continue
    m = re.match(r"\s+(SQ_\w+|FETCH_SIZE)\s+(\S+)", line)
    if m and kern:
        cur[m.group(1)] = float(m.group(2))
keys = ["SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_ACTIVE_INST_LDS", "SQ_LDS_BANK_CONFLICT", "SQ_WAIT_ANY", "SQ_WAVE_CYCLES",
        "FETCH_SIZE"]
# FETCH_SIZE (PHASE_FETCH=1 runs) is in KiB; x 1.994, the factor tools/pmc_traffic.py calibrates on the
# prep-only build (whose reads are exactly the input bytes + offsets)
FETCH_FACTOR = 1.994
print("%-24s %7s %7s | %8s %8s %9s %9s %6s %8s %9s" % ("phase (build)", "ms", "+ms", "+VALU G", "+LDS G", "+LDSact G",
                                                          "+LDScnf G", "ratio", "+wait G", "+read MB"))
prev = {k: 0.0 for k in keys}
prev_ms = 0.0
for b in order:
    r = rows.get(b)
    if not r:
        continue
    ms = r.get("ns", 0.0) / 1e6
    d = {k: r.get(k, 0.0) - prev[k] for k in keys}
    act, cnf = d["SQ_ACTIVE_INST_LDS"], d["SQ_LDS_BANK_CONFLICT"]
    rd = ("%9.1f" % (d["FETCH_SIZE"] * 1024 * FETCH_FACTOR / 1e6)) if "FETCH_SIZE" in r else "        -"
    print("%-24s %7.3f %7.3f | %8.3f %8.3f %9.3f %9.3f %6.2f %8.3f %s" % (
        names.get(b, b), ms, ms - prev_ms, d["SQ_INSTS_VALU"] / 1e9, d["SQ_INSTS_LDS"] / 1e9, act / 1e9, cnf / 1e9,
        cnf / act if act > 0 else 0.0, d["SQ_WAIT_ANY"] / 1e9, rd))
    prev = {k: r.get(k, 0.0) for k in keys}
    prev_ms = ms
full = rows.get("dptok")
if full and full.get("SQ_ACTIVE_INST_LDS"):
    print("full kernel: LDS conflict cycles / active LDS cycles = %.2f" % (full["SQ_LDS_BANK_CONFLICT"] / full["SQ_ACTIVE_INST_LDS"]))
