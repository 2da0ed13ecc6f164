"""Diagnostic (GPU box): the first pass's per-wave timeline at several call sizes (libdpt_stamps.so build).

    python tools/wave_timeline.py [ascii|s2orc] n1 n2 ...        (default: ascii 125000 250000 1000000)

Every wave of the persistent grid stamps s_memrealtime (100 MHz, one clock for the chip) at its first
instruction, at the end of each slot round (with the round's busy slots) and at its exit (WST_REC in
dpt_kernels.hip).  Per call size this splits the pass's span T into
  ramp   mean over waves of (first instruction - the grid's first instruction)
  tail   mean over waves of (the grid's last exit - the wave's exit)
  work   the rest (mean wave span), and the work into its rounds: mean duration of round k, of rounds with
         4 / 3 / 2 / 1 busy slots, of each wave's last round,
and reports the time per 4-string round of work (work x waves / (strings / 4)) against the largest call's.
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("DPT_LIB", os.path.join(ROOT, "ablibs/libdpt_wstamps.so"))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dp-tokenization_amd")]
import numpy as np  # noqa: E402

from dptok import Encoder, Vocab, synth, _lib  # noqa: E402


def analyse(w, n_str):
    TICK_US = 0.01   # 100 MHz
    nw = int(np.count_nonzero(w[:, 0]))
    w = w[:nw]
    entry = w[:, 0].astype(np.int64)
    last = w[:, -1]
    exit_ = (last & ((1 << 48) - 1)).astype(np.int64)
    rounds = (last >> 48).astype(np.int64)
    t0, t1 = entry.min(), exit_.max()
    T = (t1 - t0) * TICK_US
    ramp = float((entry - t0).mean()) * TICK_US
    tail = float((t1 - exit_).mean()) * TICK_US
    span = float((exit_ - entry).mean()) * TICK_US
    # rounds: end times and busy slots
    R = w.shape[1] - 3
    claims = w[:, -2].astype(np.int64)
    ends = (w[:, 1:1 + R] & ((1 << 56) - 1)).astype(np.int64)
    busy = (w[:, 1:1 + R] >> 56).astype(np.int64)
    by_k, by_busy, last_round, last_start = {}, {1: [], 2: [], 3: [], 4: []}, [], []
    last_end = np.zeros(nw, dtype=np.int64)
    for i in range(nw):
        prev = entry[i]
        nr = min(int(rounds[i]), R)   # (every recorded round had busy slots; the final, empty one is not recorded)
        for k in range(nr):
            dur = (ends[i, k] - prev) * TICK_US
            by_k.setdefault(k, []).append(dur)
            by_busy.setdefault(int(busy[i, k]), []).append(dur)
            if k == nr - 1:
                last_round.append(dur)
                last_start.append((prev - t0) * TICK_US)
            prev = ends[i, k]
        last_end[i] = prev
    out = {
        "strings": n_str, "waves": nw, "span_us": round(T, 2),
        "ramp_us": round(ramp, 2), "ramp_max_us": round(float((entry - t0).max()) * TICK_US, 2),
        "tail_us": round(tail, 2), "mean_wave_span_us": round(span, 2),
        "busy_frac": round(span / T, 4),
        "rounds_per_wave": round(float(rounds.mean()), 3),
        "round_us_by_index": {k: round(float(np.mean(v)), 2) for k, v in sorted(by_k.items()) if k < 8 or k % 8 == 0},
        "round_us_by_busy": {b: [len(v), round(float(np.mean(v)), 2) if v else None] for b, v in sorted(by_busy.items())},
        "last_round_us": round(float(np.mean(last_round)), 2) if last_round else None,
        "last_round_start_us_pct5_50_95_100": [round(float(np.percentile(last_start, q)), 2) for q in (5, 50, 95, 100)] if last_start else None,
        "claims_per_wave_mean_max": [round(float(claims.mean()), 2), int(claims.max())],
        "exit_after_last_round_us": round(float(np.mean(exit_ - last_end)) * TICK_US, 2),
    }
    full = sum(len(v) * np.mean(v) for v in by_busy.values() if v)
    out["work_us_per_4string_round"] = round(float(full) / (n_str / 4.0), 4)
    return out


def main():
    gen = sys.argv[1] if len(sys.argv) > 1 and not sys.argv[1].isdigit() else "ascii"
    sizes = [int(x) for x in sys.argv[1:] if x.isdigit()] or [125000, 250000, 1000000]
    enc = Encoder(Vocab(synth.llama_shaped_vocab(), 0))
    lib = _lib.lib()
    lib.dpt_debug_wstamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    maxw, nn = ctypes.c_uint(), ctypes.c_uint()
    lib.dpt_debug_wstamps_dims(ctypes.byref(maxw), ctypes.byref(nn))
    buf = np.zeros((maxw.value, nn.value), dtype=np.uint64)
    for n in sizes:
        if gen == "ascii":
            text, offs = synth.random_ascii_corpus(n, 256, seed=1)
        else:
            text, offs = synth.s2orc_like_corpus(n, seed=4)
        import torch
        dev = torch.device("cuda", 0)
        dt = torch.from_numpy(text).to(dev)
        do = torch.from_numpy(offs.view(np.int64)).to(dev)
        nb = int(offs[-1])
        ids = torch.empty(nb + n, dtype=torch.int32, device=dev)
        io = torch.empty(n + 1, dtype=torch.int64, device=dev)
        st = torch.empty(n, dtype=torch.int32, device=dev)
        stream = torch.cuda.current_stream(dev).cuda_stream

        def run():
            enc.encode_device(dt.data_ptr(), nb, do.data_ptr(), n, ids.data_ptr(), nb + n, io.data_ptr(), st.data_ptr(),
                              stream=stream)
        res = []
        for rep in range(4):
            run()
            torch.cuda.synchronize()
            lib.dpt_debug_wstamps(None, 1)
            run()
            torch.cuda.synchronize()
            lib.dpt_debug_wstamps(buf.ctypes.data, 0)
            if rep:
                res.append(analyse(buf.copy(), n))
        best = min(res, key=lambda r: r["span_us"])
        best["gen"] = gen
        print(json.dumps(best), flush=True)


if __name__ == "__main__":
    main()
