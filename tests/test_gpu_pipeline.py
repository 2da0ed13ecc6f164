"""Pipelined device calls (round 4, dpt_ctx_pipeline / dpt_ctx_join) and the LDS-free CSR pass they use
(finish_lite_kernel: one wave per 256-string batch, chunks of <= 64 ids, the histogram by one atomic per
distinct count).  Every call's CSR ids, offsets, statuses and DPT_HIST_OVERWRITE histogram are checked
against the C oracle / a CPU count:
  * the lite pass alone (DPT_LITE=1, ordinary calls) on the fold and scan prefix paths, short and
    multi-window strings, strings without ids (status 1 / 2) and the int32 staging of the toy vocabulary;
  * a sequence of pipelined calls of changing sizes (the two workspace sets grow while the other one's
    CSR pass may still run), each into its own output buffers, checked only after one join."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

FIN_BATCH, FIN_FOLD_MAX = 256, 2048   # dpt_internal.h
N_BINS = 64


def _pack(texts):
    from dptok import pack_strings
    return pack_strings(texts)


def _inputs(n, seed, kind):
    from dptok import synth
    rng = np.random.default_rng(seed)
    if kind == "ascii":
        return synth.random_ascii_corpus(n, 200, seed=seed)
    if kind == "long":   # multi-window strings (chunks of many strings' ids per round)
        words = ["".join(chr(c) for c in rng.integers(0x61, 0x7B, size=int(rng.integers(1, 12)))) for _ in range(4000)]
        texts = [" ".join(rng.choice(words, size=int(rng.integers(1, 700)))) for _ in range(n)]
        return _pack(texts)
    pool = [chr(c) for c in range(0x21, 0x7F)] + ["é", "中", "\n", " "] * 3   # statuses 1 / 2 with the toy vocab
    texts = ["" if k % 9 == 0 else "".join(rng.choice(pool, size=int(rng.integers(1, 300)))) for k in range(n)]
    return _pack(texts)


def _device_call(torch, enc, text, offs, s, hist=None):
    n = len(offs) - 1
    dt = torch.from_numpy(np.ascontiguousarray(text)).cuda()
    do = torch.from_numpy(np.ascontiguousarray(offs).view(np.int64)).cuda()
    ids = torch.empty(max(len(text), 1), dtype=torch.int32, device="cuda")
    id_off = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    st = torch.empty(max(n, 1), dtype=torch.int32, device="cuda")
    if hist is None:
        hist = torch.full((N_BINS + 8,), -3, dtype=torch.int64, device="cuda")
    enc.set_histogram(hist.data_ptr(), N_BINS, overwrite=True)
    enc.encode_device(dt.data_ptr(), len(text), do.data_ptr(), n, ids.data_ptr(), max(len(text), 1),
                      id_off.data_ptr(), st.data_ptr(), stream=s)
    return (dt, do, ids, id_off, st, hist)


def _check(orc, text, offs, res, what):
    _, _, ids, id_off, st, hist = res
    n = len(offs) - 1
    rids, roff, rst, _ = orc.encode_csr(text, offs)
    off_h = id_off.cpu().numpy().view(np.uint64)
    assert np.array_equal(off_h, roff), what
    assert np.array_equal(ids[: int(off_h[-1])].cpu().numpy(), rids), what
    assert np.array_equal(st[:n].cpu().numpy(), rst), what
    counts = np.diff(roff.astype(np.int64))
    h = hist.cpu().numpy()
    assert h[N_BINS] == counts.sum() and h[N_BINS + 1] == n, (what, h[N_BINS:])
    want = np.bincount(np.minimum(counts, N_BINS - 1), minlength=N_BINS)
    assert np.array_equal(h[:N_BINS], want), what
    assert np.array_equal(h[N_BINS + 2:N_BINS + 7], np.bincount(np.minimum(rst, 4), minlength=5)), what


@pytest.mark.parametrize("kind,n", [("ascii", 3000), ("ascii", FIN_BATCH * FIN_FOLD_MAX + 900), ("long", 700),
                                    ("toy", 5000)])
def test_lite_csr_pass(vocabs, kind, n):
    torch = pytest.importorskip("torch")
    from dptok import Encoder, Vocab
    from oracle import oracle
    t2i = vocabs["toy1k" if kind == "toy" else "llama32k"]
    enc, orc = Encoder(Vocab(t2i, 0)), oracle.OracleVocab(t2i)
    text, offs = _inputs(n, 7, kind)
    s = torch.cuda.current_stream().cuda_stream
    old = os.environ.get("DPT_LITE")
    os.environ["DPT_LITE"] = "1"
    try:
        res = _device_call(torch, enc, text, offs, s)
        torch.cuda.synchronize()
    finally:
        if old is None:
            os.environ.pop("DPT_LITE", None)
        else:
            os.environ["DPT_LITE"] = old
    _check(orc, text, offs, res, (kind, n))


def test_pipelined_calls(vocabs):
    torch = pytest.importorskip("torch")
    from dptok import Encoder, Vocab
    from oracle import oracle
    t2i = vocabs["llama32k"]
    enc, orc = Encoder(Vocab(t2i, 0)), oracle.OracleVocab(t2i)
    csr = torch.cuda.Stream()
    enc.pipeline(csr.cuda_stream)
    s = torch.cuda.current_stream().cuda_stream
    plan = [("ascii", 20000, 1), ("ascii", 20000, 2), ("long", 300, 3), ("ascii", 3000, 4),
            ("ascii", FIN_BATCH * FIN_FOLD_MAX + 300, 5), ("ascii", 100, 6), ("ascii", 40000, 7), ("ascii", 257, 8)]
    done = []
    try:
        for kind, n, seed in plan:
            text, offs = _inputs(n, seed, kind)
            done.append((text, offs, _device_call(torch, enc, text, offs, s), (kind, n, seed)))
        enc.join(s)
        torch.cuda.synchronize()
    finally:
        enc.pipeline(0)
    for text, offs, res, what in done:
        _check(orc, text, offs, res, what)
    # ordinary calls again on the same context
    text, offs = _inputs(5000, 11, "ascii")
    res = _device_call(torch, enc, text, offs, s)
    torch.cuda.synchronize()
    _check(orc, text, offs, res, "after")


def test_pipelined_calls_one_histogram(vocabs):
    """Every pipelined call arms the SAME histogram buffer (DPT_HIST_OVERWRITE): each call's zeroing is
    ordered after the previous call's CSR pass, so after the join it holds the last call's counts."""
    torch = pytest.importorskip("torch")
    from dptok import Encoder, Vocab
    from oracle import oracle
    t2i = vocabs["llama32k"]
    enc, orc = Encoder(Vocab(t2i, 0)), oracle.OracleVocab(t2i)
    csr = torch.cuda.Stream()
    enc.pipeline(csr.cuda_stream)
    s = torch.cuda.current_stream().cuda_stream
    hist = torch.full((N_BINS + 8,), -3, dtype=torch.int64, device="cuda")
    keep = []
    try:
        for k, n in enumerate([30000, 3000, 30000, 600, 20000]):
            text, offs = _inputs(n, 40 + k, "ascii")
            keep.append((text, offs, _device_call(torch, enc, text, offs, s, hist=hist)))
        enc.join(s)
        torch.cuda.synchronize()
    finally:
        enc.pipeline(0)
    for text, offs, res in keep:   # every call's CSR arrays
        _, _, ids, id_off, st, _ = res
        rids, roff, rst, _ = orc.encode_csr(text, offs)
        assert np.array_equal(id_off.cpu().numpy().view(np.uint64), roff)
        assert np.array_equal(ids[: int(roff[-1])].cpu().numpy(), rids)
    text, offs, _ = keep[-1]
    counts = np.diff(orc.encode_csr(text, offs)[1].astype(np.int64))
    h = hist.cpu().numpy()
    assert np.array_equal(h[:N_BINS], np.bincount(np.minimum(counts, N_BINS - 1), minlength=N_BINS))
    assert h[N_BINS] == counts.sum() and h[N_BINS + 1] == len(counts)
