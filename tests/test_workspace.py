"""Workspace bounds and the unbounded pass's arena.

The device path's workspace is the staged ids (2 bytes per input byte for int16-range vocabularies),
16 bytes per string and the unbounded pass's arena -- 20 bytes per input byte of the strings routed
to it, sized by default to max(4 MiB, n_bytes/32) input bytes -- not 16 + 4 + 2 bytes per input
byte of the whole batch as in round 1.  A batch whose long-word strings exceed the arena gets status
3 for those strings on the device path (the caller reads dpt_ctx_long_need, reserves and reruns);
the host path does that itself, so it stays exact for any length.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_workspace_at_cfg2_is_under_3x_input(vocabs):
    from dptok import Encoder, Vocab
    enc = Encoder(Vocab(vocabs["llama32k"], 0))
    n_str, n_bytes = 1_000_000, 256_000_000
    enc.reserve(n_bytes, n_str)
    dev, _ = enc.workspace_bytes()
    assert dev <= 3 * n_bytes, dev / n_bytes


def _long_batch(rng, n=40, L=200_000):
    # single-word strings of L random printable bytes: every one goes to the unbounded pass
    return ["".join(chr(c) for c in rng.integers(0x21, 0x7F, size=L)) for _ in range(n)]


def test_arena_overflow_device_path_then_reserve(vocabs):
    torch = pytest.importorskip("torch")
    from dptok import Encoder, Vocab, pack_strings
    from oracle import oracle
    rng = np.random.default_rng(3)
    texts = _long_batch(rng) + ["short one", "ab cd"]
    text, offs = pack_strings(texts)
    n, nb = len(texts), int(offs[-1])
    enc = Encoder(Vocab(vocabs["llama32k"], 0))
    dt = torch.from_numpy(np.array(text)).cuda()
    do = torch.from_numpy(offs.view(np.int64)).cuda()
    ids = torch.empty(nb, dtype=torch.int32, device="cuda")
    io = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    st = torch.empty(n, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream().cuda_stream

    def run():
        enc.encode_device(dt.data_ptr(), nb, do.data_ptr(), n, ids.data_ptr(), nb, io.data_ptr(), st.data_ptr(), stream=s)
        torch.cuda.synchronize()
        return st.cpu().numpy(), io.cpu().numpy().view(np.uint64), ids.cpu().numpy()

    status, _, _ = run()
    need, cap = enc.long_need()
    assert need == 40 * 200_000 and cap < need          # default arena: 4 MiB of the 8 MB routed there
    assert (status == 3).sum() > 0 and status[-1] == 0 and status[-2] == 0
    enc.reserve(nb, n, long_bytes=need)
    status, off_h, ids_h = run()
    rids, roff, rst, _ = oracle.OracleVocab(vocabs["llama32k"]).encode_csr(text, offs)
    assert np.array_equal(status, rst) and np.array_equal(off_h, roff)
    assert np.array_equal(ids_h[: int(roff[-1])], rids)


def test_arena_overflow_host_path_reruns(vocabs):
    from dptok import Encoder, Vocab, pack_strings
    from oracle import oracle
    rng = np.random.default_rng(4)
    # long strings interleaved with short ones: only the long ones overflow and run again, and
    # their ids are spliced between the short strings' (dpt_api.cpp rerun_too_long)
    texts = []
    for k, t in enumerate(_long_batch(rng, n=30)):
        texts += [t, "x y z" if k % 2 else "", " ab\ncd"]
    text, offs = pack_strings(texts)
    enc = Encoder(Vocab(vocabs["llama32k"], 0))
    got = enc.encode_csr(text, offs)
    ref = oracle.OracleVocab(vocabs["llama32k"]).encode_csr(text, offs)
    for a, b in zip(got[:3], ref[:3]):
        assert np.array_equal(a, b)
    need, cap = enc.long_need()
    # the last call reran only the strings the default 4 MiB arena could not hold (20 of 30 fitted)
    assert need == 10 * 200_000 <= cap


def test_reserved_arena_is_not_resized_by_encode(vocabs):
    """An explicitly reserved arena stays as reserved on the device path (no reallocation inside a
    reserved call: capture-safe), even when the call's default would be larger."""
    torch = pytest.importorskip("torch")
    from dptok import Encoder, Vocab, synth
    enc = Encoder(Vocab(vocabs["llama32k"], 0))
    text, offs = synth.random_ascii_corpus(200_000, 256, seed=2)   # default arena: max(4 MiB, n_bytes/32) > 1 MiB
    n, nb = len(offs) - 1, int(offs[-1])
    enc.reserve(nb, n, long_bytes=1 << 20)
    _, cap0 = enc.long_need()
    dt = torch.from_numpy(text).cuda()
    do = torch.from_numpy(offs.view(np.int64)).cuda()
    ids = torch.empty(nb, dtype=torch.int32, device="cuda")
    io = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    st = torch.empty(n, dtype=torch.int32, device="cuda")
    enc.encode_device(dt.data_ptr(), nb, do.data_ptr(), n, ids.data_ptr(), nb, io.data_ptr(), st.data_ptr(),
                      stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    need, cap1 = enc.long_need()
    assert cap1 == cap0 and need == 0
    assert (st.cpu().numpy() == 0).all()
