"""Interleaved in-process A/B of libdpt.so builds (GPU box).

    python tools/ab_inproc.py <workload> <n_strings> <rounds> lib1.so lib2.so ...

workload: ascii (cfg2), s2orc (cfg4), arabic (cfg5), bloom; ascii_p / s2orc_p: llama mode (cfg2p / cfg4p);
short: 1..12-byte strings (per-word calls).  The corpus is generated and uploaded
ONCE; every library gets its own vocab + ctx (ctypes.CDLL: each build's kernels in their own
namespace, one HIP runtime -- torch's); each round times K encodes of every library back to back
(HIP events on the stream), so drift of the box hits all of them alike.  Outputs of every library
must equal the first one's (ids, offsets, status), else the run fails.  Prints one line per library:
median / min ms per encode and GB/s over the corpus bytes.
"""
import ctypes
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dp-tokenization_amd")]
import numpy as np  # noqa: E402

from dptok import synth  # noqa: E402


def corpus(gen, n):
    cut = None
    if gen == "bloom":
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        from bloom_fixture import big_vocab
        t2i = big_vocab()
        text, offs, cut = synth.bloom_like_parallel(n, t2i, procs=16, length=256)
    else:
        t2i = synth.llama_shaped_vocab()
        if gen.endswith("_p"):   # llama mode (PRESPLIT): the same corpus pre-split as bench.py's cfg2p / cfg4p
            _, text, offs, _ = corpus(gen[:-2], n)
            text, offs, cut = synth.llama_words(text, offs)
            return t2i, text, offs, cut
        if gen == "short":   # per-word-sized strings: 1..12 random printable bytes (a few ids each)
            rng = np.random.default_rng(3)
            lens = rng.integers(1, 13, n)
            offs = np.zeros(n + 1, dtype=np.uint64)
            offs[1:] = np.cumsum(lens)
            text = rng.integers(0x20, 0x7F, int(offs[-1])).astype(np.uint8)
            return t2i, text, offs, None
        if gen == "ascii":
            text, offs = synth.random_ascii_corpus(n, 256, seed=1)
        elif gen == "s2orc":
            text, offs = synth.generate_parallel("s2orc", n, procs=16, seed=4)
        else:
            text, offs = synth.generate_parallel("arabic", n, procs=16, length=256, seed=5)
    return t2i, text, offs, cut


def main():
    gen, n, rounds = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    libs = sys.argv[4:]
    t2i, text, offs, cut = corpus(gen, n)   # (forks before the GPU is touched)
    import torch
    from dptok.engine import encode_utf8
    P = ctypes.c_void_p
    dev = torch.device("cuda", 0)
    nb = int(offs[-1])
    dt = torch.from_numpy(text).to(dev)
    do = torch.from_numpy(offs.view(np.int64)).to(dev)
    dc = torch.from_numpy(cut).to(dev) if cut is not None else None
    mode = (1 if gen.endswith("_p") else 2) if cut is not None else 0
    toks = list(t2i.keys())
    encs = [encode_utf8(t) for t in toks]
    boff = np.zeros(len(encs) + 1, dtype=np.uint64)
    boff[1:] = np.cumsum([len(e) for e in encs], dtype=np.uint64)
    blob = np.frombuffer(b"".join(encs) + b"\0", dtype=np.uint8)
    bids = np.array([t2i[t] for t in toks], dtype=np.int32)
    stream = torch.cuda.current_stream(dev).cuda_stream
    runs = []
    # per-library switches (comma lists, one entry per library): AB_HIST=1 folds the 258-bin token
    # histogram into every encode (DPT_HIST_OVERWRITE, as bench.py's step), AB_PROF=1 turns the
    # context's stage profiling on (bench.py's events around the passes)
    hist_on = [x == "1" for x in os.environ.get("AB_HIST", "").split(",")] if os.environ.get("AB_HIST") else []
    prof_on = [x == "1" for x in os.environ.get("AB_PROF", "").split(",")] if os.environ.get("AB_PROF") else []
    hists = []
    for li, path in enumerate(libs):
        L = ctypes.CDLL(os.path.abspath(path))
        L.dpt_vocab_create.argtypes = [P, P, P, ctypes.c_uint32, ctypes.c_int, ctypes.POINTER(P)]
        L.dpt_ctx_create.argtypes = [ctypes.c_int, ctypes.POINTER(P)]
        L.dpt_ctx_reserve_vocab.argtypes = [P, P, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64]
        L.dpt_encode.argtypes = [P, P, ctypes.c_int, P, ctypes.c_uint64, P, P, ctypes.c_uint64, P, ctypes.c_uint64, P, P, P, P]
        L.dpt_last_error.restype = ctypes.c_char_p
        v, c = P(), P()
        assert L.dpt_vocab_create(blob.ctypes.data, boff.ctypes.data, bids.ctypes.data, len(boff) - 1, 0, ctypes.byref(v)) == 0, L.dpt_last_error()
        assert L.dpt_ctx_create(0, ctypes.byref(c)) == 0
        assert L.dpt_ctx_reserve_vocab(c, v, nb, n, 0) == 0
        hp = None
        if li < len(hist_on) and hist_on[li]:
            h = torch.zeros(258 + 8, dtype=torch.int64, device=dev)
            hists.append(h)
            hp = P(h.data_ptr())
            L.dpt_ctx_set_histogram_ex.argtypes = [P, P, ctypes.c_uint32, ctypes.c_int]
        if li < len(prof_on) and prof_on[li]:
            L.dpt_ctx_profile.argtypes = [P, ctypes.c_int]
            assert L.dpt_ctx_profile(c, 1) == 0
        ids = torch.empty(nb, dtype=torch.int32, device=dev)
        io = torch.empty(n + 1, dtype=torch.int64, device=dev)
        st = torch.empty(n, dtype=torch.int32, device=dev)

        def enc(L=L, v=v, c=c, ids=ids, io=io, st=st, hp=hp):
            if hp is not None:
                assert L.dpt_ctx_set_histogram_ex(c, hp, 258, 1) == 0
            rc = L.dpt_encode(c, v, mode, P(dt.data_ptr()), nb, P(do.data_ptr()), P(dc.data_ptr() if dc is not None else None), n,
                              P(ids.data_ptr()), nb, P(io.data_ptr()), P(st.data_ptr()), None, P(stream))
            assert rc == 0, L.dpt_last_error()
        for _ in range(3):
            enc()
        torch.cuda.synchronize()
        runs.append({"path": path, "enc": enc, "ids": ids, "io": io, "st": st, "ms": []})
    ref = runs[0]
    for r in (runs[1:] if os.environ.get("AB_NOCHECK") != "1" else []):
        same = torch.equal(r["io"], ref["io"]) and torch.equal(r["st"], ref["st"]) and \
            torch.equal(r["ids"][: int(ref["io"][-1].item())], ref["ids"][: int(ref["io"][-1].item())])
        if not same:
            raise SystemExit("ab_inproc: %s differs from %s" % (r["path"], ref["path"]))
    K = 5
    for _ in range(rounds):
        for r in runs:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(K):
                r["enc"]()
            e1.record()
            e1.synchronize()
            r["ms"].append(e0.elapsed_time(e1) / K)
    for r in runs:
        med = statistics.median(r["ms"])
        print("%-40s median %.4f ms  min %.4f ms  %.2f GB/s  (%d rounds)" % (r["path"], med, min(r["ms"]), nb / med / 1e6, rounds),
              flush=True)


if __name__ == "__main__":
    main()
