"""Phase table from a tools/gpu_phase_wl.sh log: per stop build, the tokenize kernel's time and counters,
and the phase increments (ms) between consecutive builds."""
import re, sys
names = {"var_stop1": "prep", "var_stop21": "+A0", "var_stop2": "+A walk", "var_stop25": "+B cuts",
         "var_stop26": "+B recurrence", "var_stop27": "+B transfer/fixup", "var_stop3": "+C0/C1", "dptok": "+C2 (full)"}
rows, cur, kern = [], None, False
for line in open(sys.argv[1]):
    m = re.match(r"== (\S+)", line)
    if m:
        cur = {"tag": m.group(1)}; rows.append(cur); kern = False
        continue
    if "tokenize_kernel<256" in line and cur is not None:
        kern = True
        cur["ns"] = float(line.split("avg_ns=")[1])
        continue
    if "tokenize_kernel<2048" in line:
        kern = False
        continue
    m = re.match(r"\s+(SQ_\w+)\s+(\S+)", line)
    if m and kern:
        cur[m.group(1)] = float(m.group(2))
prev = 0.0
print("%-22s %8s %8s %9s %9s %9s %10s" % ("build", "ms", "+ms", "VALU(G)", "SALU(G)", "LDS(G)", "LDSconf(G)"))
for r in rows:
    ms = r.get("ns", 0) / 1e6
    print("%-22s %8.3f %8.3f %9.3f %9.3f %9.3f %10.3f" % (names.get(r["tag"], r["tag"]), ms, ms - prev, r.get("SQ_INSTS_VALU", 0) / 1e9,
                                                r.get("SQ_INSTS_SALU", 0) / 1e9, r.get("SQ_INSTS_LDS", 0) / 1e9,
                                                r.get("SQ_LDS_BANK_CONFLICT", 0) / 1e9))
    prev = ms
