"""Reads a rocprofv3 kernel trace (run_kernel_trace.csv) of `bench.py` with two batches in flight and reports how
the consecutive calls' kernels overlap: per first-pass launch, the time it started before the previous call's
finish pass ended (and before the previous first pass ended), and the GPU-busy span against the summed kernel
durations.

    python tools/overlap_trace.py <run_kernel_trace.csv>
"""
import csv
import sys


def main():
    rows = []
    for r in csv.DictReader(open(sys.argv[1])):
        name = r.get("Kernel_Name", "")
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
    rows.sort()
    tok = [(s, e) for s, e, n in rows if "tokenize_kernel<256" in n]
    fin = [(s, e) for s, e, n in rows if "finish_kernel" in n]
    ov_fin, ov_tok = [], []
    for k in range(1, len(tok)):
        s = tok[k][0]
        prev_f = [e for (fs, e) in fin if fs < s]
        if prev_f:
            ov_fin.append(max(0, max(prev_f) - s) / 1e3)
        ov_tok.append(max(0, tok[k - 1][1] - s) / 1e3)
    span = (rows[-1][1] - rows[0][0]) / 1e3
    busy = sum(e - s for s, e, _ in rows) / 1e3
    print("first-pass launches %d; mean us a first pass started before the previous finish pass ended: %.1f; "
          "before the previous first pass ended: %.1f; kernel time %.0f us in a span of %.0f us (x%.2f)"
          % (len(tok), sum(ov_fin) / max(len(ov_fin), 1), sum(ov_tok) / max(len(ov_tok), 1), busy, span, busy / span))


if __name__ == "__main__":
    main()
