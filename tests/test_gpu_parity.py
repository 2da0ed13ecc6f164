"""GPU parity: the HIP engine (through the C-ABI) against the reference's golden
vectors (bit-exact ids + status + capped lengths) and against the C oracle on
seeded random inputs at larger sizes."""
import numpy as np
import pytest

from conftest import CORPUS_FIXTURES, load_golden

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engines(vocabs):
    from dptok import Encoder, Vocab
    return {k: Encoder(Vocab(v, 0)) for k, v in vocabs.items()}


@pytest.fixture(scope="module")
def oracles(vocabs):
    from oracle import oracle
    return {k: oracle.OracleVocab(v) for k, v in vocabs.items()}


def test_token_hash_tables_build(engines):
    """C2's token hash exists for both test vocabularies (dpt_vocab_stats, ABI 2), as a two-choice
    table: a lookup visits a key's home bucket and its partner, never a probe chain (round 5)."""
    for k, e in engines.items():
        st = e.vocab.stats
        assert st["hash_max_probe"] == 2 and st["hash_buckets"] >= st["n_tokens"] // 2, (k, st)


def _csr(texts):
    from dptok import pack_strings
    return pack_strings(texts)


def _cmp_csr(a, b):
    ids_a, off_a, st_a = a[:3]
    ids_b, off_b, st_b = b[:3]
    assert np.array_equal(st_a, st_b), np.nonzero(st_a != st_b)[0][:10]
    assert np.array_equal(off_a, off_b), np.nonzero(off_a != off_b)[0][:10]
    assert np.array_equal(ids_a, ids_b)


@pytest.mark.parametrize("name", CORPUS_FIXTURES)
def test_golden_vectors(name, engines):
    g = load_golden(name)
    cases = [c for c in g["cases"] if not c.get("skipped")]
    text, offs = _csr([c["text"] for c in cases])
    ids, id_off, st, capped = engines[g["vocab"]].encode_csr(text, offs)
    for i, c in enumerate(cases):
        got = ids[int(id_off[i]):int(id_off[i + 1])].tolist()
        assert int(st[i]) == c["status"], (i, c["text"][:50])
        assert got == c["ids"], (i, c["text"][:50])
        if c.get("capped") is not None:
            assert int(capped[i]) == c["capped"], (i, c["text"][:50])


def test_small_random_vocab_cases():
    from dptok import Encoder, Vocab
    g = load_golden("small_random.json.gz")
    bad = []
    for c in g["cases"]:
        t2i = {t: i for i, t in enumerate(c["vocab"])}
        (ids, st), = Encoder(Vocab(t2i, 0)).encode_strs([c["text"]])
        if (ids, st) != (c["ids"], c["status"]):
            bad.append((c["text"], c["vocab"], ids, st, c["ids"], c["status"]))
    assert not bad, bad[:3]


@pytest.mark.parametrize("n,length,seed", [(131072, 256, 7), (20000, 64, 3), (4096, 1000, 9)])
def test_random_ascii_vs_oracle(n, length, seed, engines, oracles):
    from dptok import synth
    text, offs = synth.random_ascii_corpus(n, length, seed=seed)
    got = engines["llama32k"].encode_csr(text, offs)
    ref = oracles["llama32k"].encode_csr(text, offs)
    _cmp_csr(got, ref)
    assert np.array_equal(got[3], ref[3])


def test_s2orc_and_arabic_vs_oracle(engines, oracles):
    from dptok import synth
    for text, offs in (synth.s2orc_like_corpus(600, seed=44), synth.arabic_corpus(20000, seed=55)):
        _cmp_csr(engines["llama32k"].encode_csr(text, offs), oracles["llama32k"].encode_csr(text, offs))


def test_long_words_big_window(engines, oracles):
    """Words longer than the 256-byte window take the 2048-byte pass; longer ones the unbounded
    pass (dpt_long.hip).  Every length is exact -- the reference has no length limit."""
    rng = np.random.default_rng(5)
    texts = []
    for L in (255, 256, 257, 300, 700, 1500, 2047, 2048, 2049, 3000, 5000, 20000):
        w = "".join(chr(c) for c in rng.integers(0x21, 0x7F, size=L))
        texts.append(w)
        texts.append("ab cd " + w + " ef")
        texts.append(w + " " + w[: L // 2])
        texts.append(("\n" + w[:L // 3] + " x\n").join([w[:100], w[100:]]))
    text, offs = _csr(texts)
    got = engines["llama32k"].encode_csr(text, offs)
    ref = oracles["llama32k"].encode_csr(text, offs)
    _cmp_csr(got, ref)
    assert np.array_equal(got[3], ref[3])
    assert (got[2] == 0).sum() > 0


def test_long_words_unicode_and_toy(engines, oracles):
    """The unbounded pass on multi-byte code points and on a vocabulary where many atoms are
    not tokens (capped DP, status 1), mixed with ordinary strings in one batch."""
    rng = np.random.default_rng(15)
    pool = ["é", "ß", "ع", "中", "😀", "\n", "\t", "▁"] + [chr(c) for c in range(0x21, 0x7F)] * 2
    texts = []
    for k in range(60):
        L = int(rng.integers(1, 4000)) if k % 3 else int(rng.integers(2000, 9000))
        texts.append("".join(rng.choice(pool, size=L)))
        texts.append("".join(rng.choice(pool + [" "] * 20, size=200)))
    text, offs = _csr(texts)
    for name in ("llama32k", "toy1k"):
        got = engines[name].encode_csr(text, offs)
        ref = oracles[name].encode_csr(text, offs)
        _cmp_csr(got, ref)
        assert np.array_equal(got[3], ref[3])


def test_long_pass_presplit(engines, oracles):
    """PRESPLIT strings with words longer than 2048 bytes go through the unbounded pass."""
    from oracle import oracle
    rng = np.random.default_rng(16)
    texts = ["".join(chr(c) for c in rng.integers(0x21, 0x7F, size=int(rng.integers(100, 6000)))) for _ in range(40)]
    text, offs = _csr(texts)
    cut = (rng.random(len(text)) < 0.0004).astype(np.uint8)
    got = engines["llama32k"].encode_csr(text, offs, mode="presplit", cut_mask=cut)
    ref = oracles["llama32k"].encode_csr(text, offs, mode=oracle.PRESPLIT, cut_mask=cut)
    _cmp_csr(got, ref)


def test_empty_batch_and_empty_strings(engines):
    enc = engines["llama32k"]
    ids, id_off, st, _ = enc.encode_csr(np.zeros(1, np.uint8), np.zeros(1, np.uint64))
    assert len(ids) == 0 and id_off.tolist() == [0]
    text, offs = _csr(["", "a", "", " ", ""])
    ids, id_off, st, _ = enc.encode_csr(text, offs)
    assert st.tolist() == [2, 0, 2, 1, 2]


def test_presplit_mode_vs_oracle(engines, oracles):
    from dptok import synth
    from oracle import oracle
    text, offs = synth.random_ascii_corpus(5000, 200, seed=12)
    rng = np.random.default_rng(0)
    cut = (rng.random(len(text)) < 0.12).astype(np.uint8)
    got = engines["llama32k"].encode_csr(text, offs, mode="presplit", cut_mask=cut)
    ref = oracles["llama32k"].encode_csr(text, offs, mode=oracle.PRESPLIT, cut_mask=cut)
    _cmp_csr(got, ref)


def test_device_path_and_histogram(engines, oracles):
    torch = pytest.importorskip("torch")
    from dptok import synth
    n = 50000
    text, offs = synth.random_ascii_corpus(n, 256, seed=21)
    enc = engines["llama32k"]
    dt = torch.from_numpy(text).cuda()
    do = torch.from_numpy(offs.view(np.int64)).cuda()
    ids = torch.empty(len(text), dtype=torch.int32, device="cuda")
    id_off = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    st = torch.empty(n, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    enc.encode_device(dt.data_ptr(), len(text), do.data_ptr(), n, ids.data_ptr(), len(text), id_off.data_ptr(),
                      st.data_ptr(), stream=s)
    hist = torch.zeros(258 + 8, dtype=torch.int64, device="cuda")
    enc.histogram_device(id_off.data_ptr(), st.data_ptr(), n, hist.data_ptr(), 258, stream=s)
    torch.cuda.synchronize()
    rids, roff, rst, _ = oracles["llama32k"].encode_csr(text, offs)
    off_h = id_off.cpu().numpy().view(np.uint64)
    assert np.array_equal(off_h, roff)
    assert np.array_equal(ids[: int(off_h[-1])].cpu().numpy(), rids)
    h = hist.cpu().numpy()
    counts = np.diff(roff.astype(np.int64))
    assert h[258] == counts.sum() and h[259] == n and h[260] == n
    assert np.array_equal(h[:257], np.bincount(np.minimum(counts, 257), minlength=258)[:257])


def test_device_path_output_at_high_addresses(engines, oracles):
    """The CSR ids written where a pointer's low 32 bits are >= 2^31: a 64-bit address put together
    from two readfirstlane halves sign-extends its low half unless each goes through uint32 (round 5:
    the finish copy's store resource did, and faulted the GPU)."""
    torch = pytest.importorskip("torch")
    from dptok import synth
    n = 20000
    text, offs = synth.random_ascii_corpus(n, 256, seed=23)
    enc = engines["llama32k"]
    dt = torch.from_numpy(text).cuda()
    do = torch.from_numpy(offs.view(np.int64)).cuda()
    big = torch.empty((1 << 30) + len(text), dtype=torch.int32, device="cuda")   # 4 GiB + the ids
    lo = big.data_ptr() & 0xFFFFFFFF
    e = ((0x80001000 - lo) & 0xFFFFFFFF) // 4   # the view's address has low word 0x80001000
    ids = big[e: e + len(text)]
    assert (ids.data_ptr() & 0xFFFFFFFF) >= 0x80000000
    id_off = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    st = torch.empty(n, dtype=torch.int32, device="cuda")
    enc.encode_device(dt.data_ptr(), len(text), do.data_ptr(), n, ids.data_ptr(), len(text), id_off.data_ptr(),
                      st.data_ptr(), stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    rids, roff, rst, _ = oracles["llama32k"].encode_csr(text, offs)
    off_h = id_off.cpu().numpy().view(np.uint64)
    assert np.array_equal(off_h, roff)
    assert np.array_equal(ids[: int(off_h[-1])].cpu().numpy(), rids)
    del big


@pytest.mark.parametrize("shift", [0, 1, 3])
def test_finish_one_slice_vector_copy(engines, oracles, shift):
    """Calls of >= 2048 batches (one finish block per batch, no slices, no folded prefixes: the batch-scan
    launch): the ids array `shift` ints past a 16-byte boundary, ragged strings of 0..40 bytes (many rows of the
    copy's string map cross several strings, empty strings in between), every id against the oracle."""
    torch = pytest.importorskip("torch")
    n = 600_000
    rng = np.random.default_rng(31 + shift)
    lens = rng.integers(0, 41, n)
    offs = np.zeros(n + 1, dtype=np.uint64)
    offs[1:] = np.cumsum(lens)
    text = rng.integers(0x20, 0x7F, int(offs[-1])).astype(np.uint8)
    enc = engines["llama32k"]
    dt = torch.from_numpy(text).cuda()
    do = torch.from_numpy(offs.view(np.int64)).cuda()
    buf = torch.empty(len(text) + 8, dtype=torch.int32, device="cuda")
    assert buf.data_ptr() % 16 == 0
    ids = buf[shift: shift + len(text)]
    id_off = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    st = torch.empty(n, dtype=torch.int32, device="cuda")
    enc.encode_device(dt.data_ptr(), len(text), do.data_ptr(), n, ids.data_ptr(), len(text), id_off.data_ptr(),
                      st.data_ptr(), stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    rids, roff, rst, _ = oracles["llama32k"].encode_csr(text, offs)
    off_h = id_off.cpu().numpy().view(np.uint64)
    assert np.array_equal(off_h, roff)
    assert np.array_equal(st.cpu().numpy(), rst)
    assert np.array_equal(ids[: int(off_h[-1])].cpu().numpy(), rids)


@pytest.mark.parametrize("n,n_bins", [(50000, 258), (257, 258), (100, 2), (3000, 1500), (1, 16)])
def test_histogram_folded_into_encode(n, n_bins, engines):
    """dpt_ctx_set_histogram: the finish pass's histogram (one call; n_bins > 1024 takes the separate
    pass) equals dpt_token_histogram's, statuses included (the OOV fixture's strings fail)."""
    torch = pytest.importorskip("torch")
    from dptok import synth, pack_strings
    g = load_golden("oov_llama32k.json.gz")
    texts = [c["text"] for c in g["cases"]] + synth.unpack(*synth.random_ascii_corpus(max(n, 1), 256, seed=22))
    text, offs = pack_strings(texts[:n] + ["", " "])
    m = len(offs) - 1
    enc = engines["llama32k"]
    dt = torch.from_numpy(np.array(text)).cuda()
    do = torch.from_numpy(offs.view(np.int64)).cuda()
    ids = torch.empty(len(text), dtype=torch.int32, device="cuda")
    id_off = torch.empty(m + 1, dtype=torch.int64, device="cuda")
    st = torch.empty(m, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    folded = torch.full((n_bins + 8,), 7, dtype=torch.int64, device="cuda")   # accumulated into
    sep = torch.full((n_bins + 8,), 7, dtype=torch.int64, device="cuda")
    enc.set_histogram(folded.data_ptr(), n_bins)
    enc.encode_device(dt.data_ptr(), int(offs[-1]), do.data_ptr(), m, ids.data_ptr(), len(text), id_off.data_ptr(),
                      st.data_ptr(), stream=s)
    enc.histogram_device(id_off.data_ptr(), st.data_ptr(), m, sep.data_ptr(), n_bins, stream=s)
    # one call only: the next encode adds nothing to it
    enc.encode_device(dt.data_ptr(), int(offs[-1]), do.data_ptr(), m, ids.data_ptr(), len(text), id_off.data_ptr(),
                      st.data_ptr(), stream=s)
    torch.cuda.synchronize()
    assert torch.equal(folded, sep), (folded.cpu().numpy()[-8:], sep.cpu().numpy()[-8:])
    assert int(sep[n_bins + 1]) == m + 7
    # DPT_HIST_OVERWRITE: the call's histogram replaces whatever the buffer held
    over = torch.full((n_bins + 8,), -5, dtype=torch.int64, device="cuda")
    enc.set_histogram(over.data_ptr(), n_bins, overwrite=True)
    enc.encode_device(dt.data_ptr(), int(offs[-1]), do.data_ptr(), m, ids.data_ptr(), len(text), id_off.data_ptr(),
                      st.data_ptr(), stream=s)
    torch.cuda.synchronize()
    assert torch.equal(over[: n_bins + 7], sep[: n_bins + 7] - 7), (over.cpu().numpy()[-8:], sep.cpu().numpy()[-8:])


@pytest.mark.parametrize("variant", ["rows16", "rows64"])
def test_kernel_variants_vs_oracle(variant, engines, oracles, monkeypatch):
    """Every first-pass kernel (DPT_KERNEL override) is bit-exact on cfg2 / Arabic / S2ORC samples."""
    from dptok import synth
    monkeypatch.setenv("DPT_KERNEL", variant)
    for text, offs in (synth.random_ascii_corpus(8192, 256, seed=31), synth.arabic_corpus(2048, seed=32),
                       synth.s2orc_like_corpus(200, seed=33)):
        _cmp_csr(engines["llama32k"].encode_csr(text, offs), oracles["llama32k"].encode_csr(text, offs))


def test_long_token_vocab_uses_64_lane_rows():
    """A vocabulary with tokens of 17..64 code points runs the 64-lane row kernel; still bit-exact."""
    from dptok import Encoder, Vocab, synth
    from oracle import oracle
    t2i = dict(synth.llama_shaped_vocab())
    rng = np.random.default_rng(2)
    for L in (17, 20, 24, 31, 40, 64):
        for _ in range(20):
            tok = "".join(chr(c) for c in rng.integers(0x61, 0x65, size=L))
            t2i.setdefault(tok, len(t2i))
            t2i.setdefault("▁" + tok[:-1], len(t2i))
    v = Vocab(t2i, 0)
    assert v.stats["max_cp"] > 16
    texts = ["".join(chr(c) for c in rng.integers(0x61, 0x65, size=rng.integers(1, 300))) for _ in range(3000)]
    texts += [" ".join(texts[k:k + 3]) for k in range(0, 300, 3)]
    text, offs = _csr(texts)
    _cmp_csr(Encoder(v).encode_csr(text, offs), oracle.OracleVocab(t2i).encode_csr(text, offs))


def test_mixed_unicode_vs_oracle(engines, oracles):
    """Valid UTF-8 with NUL, tabs, newlines, 2/3/4-byte code points (many outside the vocabulary,
    so the capped DP and status 1 paths run) against the C oracle, raw mode."""
    rng = np.random.default_rng(5)
    pool = ["\x00", "\t", "\n", " ", "é", "ß", "ع", "中", "文", "😀", "🤖", "▁", "<0x0A>", "<s>"] + \
           [chr(c) for c in range(0x21, 0x7F)] * 3
    texts = ["".join(rng.choice(pool, size=int(rng.integers(0, 300)))) for _ in range(6000)]
    text, offs = _csr(texts)
    for name in ("llama32k", "toy1k"):
        _cmp_csr(engines[name].encode_csr(text, offs), oracles[name].encode_csr(text, offs))


def test_atoms_mode_long_atoms():
    """ATOMS mode: atoms of up to 8 bytes are walked by the windowed kernels; a longer atom sends
    the string to the unbounded pass, which walks atoms of any length."""
    from dptok import Encoder, Vocab
    t2i = {"abcdefgh": 0, "ab": 1, "cdefgh": 2, "x": 3, "abcdefghi": 4, "i": 5, "abcdefghijklmnopqrstu": 6, "v": 7}
    enc = Encoder(Vocab(t2i, 0))
    res = enc.encode_word_atoms([[["abcdefgh", "x"]], [["ab", "cdefgh"]], [["abcdefghi"]],
                                 [["abcdefghi", "x"], ["x"]], [["abcdefghijklmnopqrstu", "v"]], [["abcdefghij"]]])
    assert res[0] == ([0, 3], 0)
    assert res[1] == ([0], 0)          # 'ab'+'cdefgh' = one token 'abcdefgh'
    assert res[2] == ([4], 0)
    assert res[3] == ([4, 3, 3], 0)
    assert res[4] == ([6, 7], 0)
    assert res[5] == ([], 1)           # one atom that is not a token: no complete tokenization


def test_tokens_longer_than_64_code_points():
    """A vocabulary with tokens of 65..300 code points: words of up to 64 atoms run in the windowed
    kernels, longer words in the unbounded pass; all exact against the oracle."""
    from dptok import Encoder, Vocab, synth
    from oracle import oracle
    t2i = dict(synth.llama_shaped_vocab())
    rng = np.random.default_rng(4)
    long_toks = []
    for L in (65, 70, 80, 150, 300):
        for _ in range(10):
            tok = "".join(chr(c) for c in rng.integers(0x61, 0x64, size=L))
            long_toks.append(tok)
            t2i.setdefault(tok, len(t2i))
    v = Vocab(t2i, 0)
    assert v.stats["max_cp"] >= 300
    short = ["".join(chr(c) for c in rng.integers(0x61, 0x64, size=rng.integers(1, 64))) for _ in range(2000)]
    short += [" ".join(short[k:k + 3]) for k in range(0, 300, 3)]
    text, offs = _csr(short)
    _cmp_csr(Encoder(v).encode_csr(text, offs), oracle.OracleVocab(t2i).encode_csr(text, offs))
    long_ = ["x" + "".join(chr(c) for c in rng.integers(0x61, 0x64, size=rng.integers(65, 400))) for _ in range(200)]
    # words that contain the long tokens verbatim, so the > 64-atom spans are taken
    for k in range(100):
        a, b = long_toks[k % len(long_toks)], long_toks[(7 * k + 3) % len(long_toks)]
        long_.append("x" + a + "ab" + b[: (k * 13) % len(b)] + " " + b)
    text, offs = _csr(long_)
    got = Encoder(v).encode_csr(text, offs)
    ref = oracle.OracleVocab(t2i).encode_csr(text, offs)
    _cmp_csr(got, ref)
    assert np.array_equal(got[3], ref[3])
    assert (got[2] == 0).sum() >= 100


def _min_tokens_bounded(atoms, vocab, max_cp, capped=False):
    """oracle/ref_port.min_tokens_for_string (inspect_tokenizer.py:77-86), or with ``capped`` the
    len_dp[-1] of ref_port.forward_dp (dp_tokenize.py:28), with spans bounded by the longest token
    (a span of L atoms has >= L code points, so longer spans are never tokens)."""
    n = len(atoms)
    best = list(range(n + 1)) if capped else [float("inf")] * (n + 1)
    best[0] = 0
    for i in range(1, n + 1):
        for j in range(max(0, i - max_cp), i):
            if best[j] + 1 < best[i] and "".join(atoms[j:i]) in vocab:
                best[i] = best[j] + 1
    return best[n]


def test_long_pass_dp_lengths(vocabs):
    """dpt_dp_host (len-only capped and uncapped) on atom lists of up to 5000 atoms: the uncapped
    minimum matches the reference's min_tokens_for_string restatement, the capped length matches
    the C oracle's capped sums through PRESPLIT."""
    from dptok import Encoder, Vocab
    from dptok.engine import atoms_to_csr
    from oracle import ref_port
    t2i = vocabs["toy1k"]
    vocab = set(t2i)
    enc = Encoder(Vocab(t2i, 0))
    max_cp = max(len(t) for t in vocab)
    rng = np.random.default_rng(17)
    letters = sorted({c for t in vocab for c in t})
    words = [list(rng.choice(letters, size=int(rng.integers(1, 60)))) for _ in range(200)]
    words += [list(rng.choice(letters, size=int(rng.integers(2000, 5000)))) for _ in range(12)]
    for w in words[:40]:
        assert _min_tokens_bounded(w, vocab, max_cp) == ref_port.min_tokens_for_string(w, vocab)
    text, offs, cut = atoms_to_csr(words)
    st, lens, _ = enc.dp(text, offs, mode="atoms", cut_mask=cut, uncapped=True)
    for k, w in enumerate(words):
        want = _min_tokens_bounded(w, vocab, max_cp)
        assert int(lens[k]) == (65535 if want == float("inf") else want), k
    for w in words[:40]:
        assert _min_tokens_bounded(w, vocab, max_cp, capped=True) == ref_port.forward_dp(w, vocab)[0][-1]
    st, lens, _ = enc.dp(text, offs, mode="atoms", cut_mask=cut)
    for k, w in enumerate(words):
        assert int(lens[k]) == _min_tokens_bounded(w, vocab, max_cp, capped=True), k


def test_tie_heavy_long_words_vs_oracle():
    """Lane-mode B + C1 (chunks cut inside words) on tie-heavy capless vocabularies over {a,b,c}:
    long words, many equal-cost tokenizations, several L*-length tokens per word (the chance-flag
    re-walk), batches that fill every row of every wave."""
    from dptok import Encoder, Vocab, pack_strings
    from oracle import oracle
    from test_lane_model import tie_heavy_case
    rng = np.random.default_rng(21)
    for _ in range(30):
        vocab, _ = tie_heavy_case(rng)
        t2i = {t: i for i, t in enumerate(vocab)}
        texts = [tie_heavy_case(rng, max_len=256)[1] for _ in range(400)]
        text, offs = pack_strings(texts)
        got = Encoder(Vocab(t2i, 0)).encode_csr(text, offs)
        ref = oracle.OracleVocab(t2i).encode_csr(text, offs)
        _cmp_csr(got, ref)
        assert np.array_equal(got[3], ref[3])


def test_ascii_windows_phase_a0(engines, oracles):
    """Pure-ASCII raw windows take phase A0 (the byte-parallel first lookup): control bytes,
    '\\n' next to spaces, runs of spaces, words cut by the 256-byte windows (later windows start
    with a space), on the 32k vocabulary (capless windows: lane-mode B/C1) and the toy vocabulary
    (many atoms are not tokens: the row recurrence), against the C oracle."""
    rng = np.random.default_rng(23)
    pool = [chr(c) for c in range(0x20, 0x7F)] * 3 + ["\n", "\t", "\x01", "\x7f", "  ", " \n", "\n "]
    texts = []
    for k in range(3000):
        n = int(rng.integers(0, 900)) if k % 4 else int(rng.integers(200, 320))
        texts.append("".join(rng.choice(pool, size=n)))
    texts += ["\n" * 300, " " * 300, "a" * 600, ("ab " * 200), "\t" * 257]
    text, offs = _csr(texts)
    for name in ("llama32k", "toy1k"):
        got = engines[name].encode_csr(text, offs)
        ref = oracles[name].encode_csr(text, offs)
        _cmp_csr(got, ref)
        assert np.array_equal(got[3], ref[3])


@pytest.mark.parametrize("seed", [31, 32])
def test_ascii_walker_and_token_hash(seed):
    """Phase A's ASCII walker (A0 slots: word starts from the '\u2581' node, the string's first atom,
    "<0x0A>" expansions at a walk's start and inside it, walks going on past A0's two-byte lookup) and
    C2's token hash (tokens of 3..16 expanded bytes with a '\u2581' prefix from a space or from the
    first atom; tokens with a newline atom and longer ones left to the walkers) on a vocabulary of
    long letter tokens and newline-bearing tokens, over multi-window strings, against the C oracle.
    Seed 32 leaves '\u2581' itself out of the vocabulary (a word start is then no token)."""
    from dptok import Encoder, Vocab, pack_strings
    from oracle import oracle
    rng = np.random.default_rng(seed)
    letters = "etaoinsh"
    vocab = set(letters) | {"\u2581" + c for c in letters} | {"<0x0A>", "\n"}
    if seed == 31:
        vocab.add("\u2581")
    for _ in range(3000):
        L = int(rng.integers(2, 17))
        w = "".join(rng.choice(list(letters), size=L))
        r = rng.random()
        if r < 0.3:
            w = "\u2581" + w[:15]
        elif r < 0.4:
            k = int(rng.integers(0, len(w)))
            w = (w[:k] + "<0x0A>" + w[k:])[:16]
        vocab.add(w)
    vocab = sorted(vocab)
    t2i = {t: i for i, t in enumerate(vocab)}
    texts = []
    for k in range(2500):
        n = int(rng.integers(1, 700))
        ch = rng.choice(list(letters) + [" "] * 2 + ["\n"] * (1 if k % 3 else 0), size=n)
        texts.append("".join(ch))
    texts += ["\n" + "etao" * 50, " " + "e" * 300, "\n\n\n", "e\ne\ne", " \nabc"]
    text, offs = pack_strings(texts)
    got = Encoder(Vocab(t2i, 0)).encode_csr(text, offs)
    ref = oracle.OracleVocab(t2i).encode_csr(text, offs)
    _cmp_csr(got, ref)
    assert np.array_equal(got[3], ref[3])


@pytest.mark.parametrize("shift", [40000, "edge"])
def test_staging_width_by_id_range(shift, vocabs):
    """Ids are staged as int16 when every id is in 0..32767 (the llama-shaped vocabularies) and as
    int32 otherwise: the same corpus through both widths -- windowed passes and the unbounded pass
    (3000-byte words) -- against the C oracle with the same ids."""
    from dptok import Encoder, Vocab, synth
    from oracle import oracle
    base = vocabs["llama32k"]
    if shift == "edge":   # the largest id is exactly 32767: still int16
        top = max(base.values())
        t2i = {t: i + (32767 - top) for t, i in base.items()}
    else:
        t2i = {t: i + shift for t, i in base.items()}
    rng = np.random.default_rng(17)
    texts = [synth.unpack(*synth.random_ascii_corpus(1, 256, seed=100 + k))[0] for k in range(64)]
    texts += ["".join(chr(c) for c in rng.integers(97, 123, size=3000)) for _ in range(8)]
    texts += ["", " ", "\n\n", "a"]
    text, offs = _csr(texts)
    got = Encoder(Vocab(t2i, 0)).encode_csr(text, offs)
    ref = oracle.OracleVocab(t2i).encode_csr(text, offs)
    _cmp_csr(got, ref)
    assert int(got[0].max()) > 32767 if shift != "edge" else int(got[0].max()) <= 32767


def test_histogram_statuses_and_overflow(engines, oracles):
    """Histogram bins with mixed statuses (empty strings: status 2) and an overflow bin (n_bins 16:
    every count >= 15 lands in bin 15), 70 001 strings (not a multiple of the block size)."""
    torch = pytest.importorskip("torch")
    from dptok import synth
    rng = np.random.default_rng(5)
    texts = synth.unpack(*synth.random_ascii_corpus(70001, 24, seed=23))
    for k in rng.choice(len(texts), 3000, replace=False):
        texts[k] = "" if k % 2 else texts[k][: int(k) % 7]
    text, offs = _csr(texts)
    n, nb = len(texts), 16
    enc = engines["llama32k"]
    dt = torch.from_numpy(np.array(text)).cuda()
    do = torch.from_numpy(offs.view(np.int64)).cuda()
    ids = torch.empty(max(len(text), 1), dtype=torch.int32, device="cuda")
    id_off = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    st = torch.empty(n, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    enc.encode_device(dt.data_ptr(), len(text), do.data_ptr(), n, ids.data_ptr(), len(text), id_off.data_ptr(),
                      st.data_ptr(), stream=s)
    hist = torch.zeros(nb + 8, dtype=torch.int64, device="cuda")
    enc.histogram_device(id_off.data_ptr(), st.data_ptr(), n, hist.data_ptr(), nb, stream=s)
    torch.cuda.synchronize()
    _, roff, rst, _ = oracles["llama32k"].encode_csr(text, offs)
    h = hist.cpu().numpy()
    counts = np.diff(roff.astype(np.int64))
    assert np.array_equal(h[:nb], np.bincount(np.minimum(counts, nb - 1), minlength=nb))
    assert h[nb] == counts.sum() and h[nb + 1] == n
    assert np.array_equal(h[nb + 2: nb + 7], np.bincount(np.clip(rst, 0, 4), minlength=5))
    assert h[nb + 4] > 0   # empty strings were counted under status 2


def test_finish_sizes_and_repeats(engines, oracles):
    """The finish pass (batch sums added by the tokenize passes, one-block scan that zeroes them and
    resets the counter block, batches split over 1..8 slices by call size) on one ctx across calls
    of changing sizes -- sums a larger earlier call left behind must never leak into this call's --
    against the C oracle."""
    torch = pytest.importorskip("torch")
    from dptok import synth
    enc = engines["llama32k"]
    s = torch.cuda.current_stream().cuda_stream
    rng = np.random.default_rng(8)
    for k, n in enumerate([70000, 1, 64, 65, 130, 4097, 70000, 3, 129]):
        lens = rng.integers(0, 300, size=n)
        texts = [synth.unpack(*synth.random_ascii_corpus(1, int(L), seed=1000 * k + i))[0] if L else "" for i, L in enumerate(lens[:64])]
        text, offs = synth.random_ascii_corpus(n, 256, seed=77 + k)
        if n > 64:   # ragged: drop a random tail of every string (empty strings included)
            cut = rng.integers(0, 257, size=n)
            parts = [text[i * 256:i * 256 + int(cut[i])].tobytes() for i in range(n)]
            offs = np.zeros(n + 1, np.uint64)
            offs[1:] = np.cumsum([len(p) for p in parts])
            text = np.frombuffer(b"".join(parts) + b"\0", np.uint8)
        else:
            text, offs = _csr(texts[:n])
        nb = int(offs[-1])
        dt = torch.from_numpy(np.array(text)).cuda()
        do = torch.from_numpy(offs.view(np.int64)).cuda()
        ids = torch.empty(max(nb, 1), dtype=torch.int32, device="cuda")
        io = torch.full((n + 1,), -7, dtype=torch.int64, device="cuda")
        st = torch.empty(n, dtype=torch.int32, device="cuda")
        enc.encode_device(dt.data_ptr(), nb, do.data_ptr(), n, ids.data_ptr(), max(nb, 1), io.data_ptr(), st.data_ptr(), stream=s)
        torch.cuda.synchronize()
        rids, roff, rst, _ = oracles["llama32k"].encode_csr(text, offs)
        off_h = io.cpu().numpy().view(np.uint64)
        assert np.array_equal(off_h, roff), (n, np.nonzero(off_h != roff)[0][:5])
        assert np.array_equal(st.cpu().numpy(), rst)
        assert np.array_equal(ids[: int(roff[-1])].cpu().numpy(), rids)


def test_finish_repeated_calls(engines, oracles):
    """4 100 calls on one ctx, with dpt_encode_padded calls (which add no batch sums) between them:
    every call's batch sums start from zero and the results stay exact."""
    torch = pytest.importorskip("torch")
    from dptok import synth
    enc = engines["toy1k"]
    n = 130
    text, offs = synth.random_ascii_corpus(n, 16, seed=5)
    nb = int(offs[-1])
    dt = torch.from_numpy(np.array(text)).cuda()
    do = torch.from_numpy(offs.view(np.int64)).cuda()
    ids = torch.empty(nb, dtype=torch.int32, device="cuda")
    io = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    st = torch.empty(n, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    rids, roff, rst, _ = oracles["toy1k"].encode_csr(text, offs)
    pids = torch.empty(nb, dtype=torch.int32, device="cuda")
    cnt = torch.empty(n, dtype=torch.int64, device="cuda")
    pst = torch.empty(n, dtype=torch.int32, device="cuda")
    for k in range(4100):
        enc.encode_device(dt.data_ptr(), nb, do.data_ptr(), n, ids.data_ptr(), nb, io.data_ptr(), st.data_ptr(), stream=s)
        if k % 7 == 3:
            enc.encode_device_padded(dt.data_ptr(), nb, do.data_ptr(), n, pids.data_ptr(), nb, cnt.data_ptr(), pst.data_ptr(), stream=s)
        if k % 512 == 0 or k >= 4090:
            torch.cuda.synchronize()
            assert np.array_equal(io.cpu().numpy().view(np.uint64), roff), k
            assert np.array_equal(ids[: int(roff[-1])].cpu().numpy(), rids), k
            assert np.array_equal(st.cpu().numpy(), rst), k


@pytest.mark.gpu
def test_enumeration_with_tokens_longer_than_64_atoms():
    """compute_shortest_tokenizations (reference dp_tokenize.py:6-70, no span limit) when optimal
    tokens span more than 64 atoms: the far predecessors come from dpt_dp_host_far's pair list, so
    the full list and its DFS order equal oracle/ref_port.enumerate_shortest (was DptError)."""
    from oracle import ref_port
    from packages.dp_tokenize import compute_shortest_tokenizations
    rng = np.random.default_rng(11)
    longs = ["".join(chr(c) for c in rng.integers(0x61, 0x64, size=L)) for L in (65, 66, 70, 80, 100, 150, 300)]
    u, w = longs[2], longs[3]
    vocab = {"a", "b", "c", "x", "ab", "bc", "ca"} | set(longs)
    vocab |= {u + w[:3], w[3:], u[:-2], u[-2:] + w}      # several far predecessors at one end
    words = [u + w, "x" + u + w, u + w + "ab", longs[0] + longs[1], longs[6] + "abc" + longs[5]]
    for k in range(25):
        a, b = longs[k % 7], longs[(3 * k + 1) % 7]
        words.append(a + "".join(chr(c) for c in rng.integers(0x61, 0x64, size=k % 6)) + b[: 60 + k])
    seen_multi = 0
    for wd in words:
        got = compute_shortest_tokenizations(list(wd), vocab, False, None)
        ref = ref_port.enumerate_shortest(list(wd), vocab)
        assert got == ref, wd[:40]
        seen_multi += len(ref[0]) > 1 and any(len(t) > 64 for tk in ref[0] for t in tk)
    got, n = compute_shortest_tokenizations(list(u + w), vocab, False, None)
    assert n == 2 and sorted(got) == sorted([[u, w], [u + w[:3], w[3:]], [u[:-2], u[-2:] + w]])
    assert seen_multi >= 5


@pytest.mark.gpu
def test_dp_host_without_far_list_reports_status_3():
    """dpt_dp_host (no far list) keeps its contract: an optimal predecessor more than 64 atoms back
    gives status 3; dpt_dp_host_far lists it instead."""
    from dptok import Encoder, Vocab
    from dptok.engine import atoms_to_csr
    rng = np.random.default_rng(12)
    t = "".join(chr(c) for c in rng.integers(0x61, 0x64, size=90))
    t2i = {"a": 0, "b": 1, "c": 2, t: 3}
    enc = Encoder(Vocab(t2i, 0))
    text, offs, cut = atoms_to_csr([list("ab" + t)])
    st, ln, ed = enc.dp(text, offs, cut_mask=cut, edges=True)
    assert int(st[0]) == 3
    st, ln, ed, far = enc.dp(text, offs, cut_mask=cut, edges=True, far=True)
    assert int(st[0]) == 0 and int(ln[0]) == 3
    assert far.tolist() == [[len(t) + 2 - 1, len(t) - 1]]


def _long_word_texts():
    """test_long_words_big_window's inputs: words of 255..20000 bytes (the 2048-byte and unbounded passes)."""
    rng = np.random.default_rng(5)
    texts = []
    for L in (255, 256, 257, 300, 700, 1500, 2047, 2048, 2049, 3000, 5000, 20000):
        w = "".join(chr(c) for c in rng.integers(0x21, 0x7F, size=L))
        texts += [w, "ab cd " + w + " ef", w + " " + w[: L // 2], ("\n" + w[:L // 3] + " x\n").join([w[:100], w[100:]])]
    return texts


@pytest.mark.parametrize("bias", [0x80000000 + 12345, (3 << 32) | 0xFFFFF000])
def test_long_pass_offsets_past_2g(bias, vocabs, oracles):
    """Round 5's fault (gpurun_out/r05v/ab_ascii_1000000.log): a 64-bit uniform value put together from two
    readfirstlane halves sign-extends an int low half >= 2^31.  Besides the finish copy's store resource
    (test_device_path_output_at_high_addresses) the fix covered the unbounded pass's arena offset and its
    far-pair base (dpt_long.hip).  dpt_ctx_debug_counter_bias starts both counters at `bias` (low word >= 2^31;
    the second also carries into the high word), so those offsets pass 2^31 without a 40-GiB arena: the
    long-word inputs (test_long_words_big_window, test_tokens_longer_than_64_code_points) through the host
    and device paths against the oracle, and the far-pair lists against an unbiased engine's."""
    torch = pytest.importorskip("torch")
    from dptok import Encoder, Vocab, synth
    from dptok.engine import atoms_to_csr
    from oracle import oracle
    # (1) the arena offset: the unbounded pass takes the words over 2048 bytes
    enc = Encoder(Vocab(vocabs["llama32k"], 0))
    enc.debug_counter_bias(bias)
    text, offs = _csr(_long_word_texts())
    ref = oracles["llama32k"].encode_csr(text, offs)
    got = enc.encode_csr(text, offs)
    _cmp_csr(got, ref)
    assert np.array_equal(got[3], ref[3])
    assert enc.long_need()[0] > 0          # (the pass ran, and the bias is subtracted from what it reports)
    n = len(offs) - 1
    dt = torch.from_numpy(text).cuda()
    do = torch.from_numpy(offs.view(np.int64)).cuda()
    ids = torch.empty(len(text), dtype=torch.int32, device="cuda")
    io = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    st = torch.empty(n, dtype=torch.int32, device="cuda")
    enc.encode_device(dt.data_ptr(), len(text), do.data_ptr(), n, ids.data_ptr(), len(text), io.data_ptr(), st.data_ptr(),
                      stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    off_h = io.cpu().numpy().view(np.uint64)
    assert np.array_equal(off_h, ref[1]) and np.array_equal(st.cpu().numpy(), ref[2])
    assert np.array_equal(ids[: int(off_h[-1])].cpu().numpy(), ref[0])
    need, cap = enc.long_need()
    assert 0 < need <= cap
    # (2) a vocabulary with tokens of 65..300 code points: words over 64 atoms take the unbounded pass
    t2i = dict(synth.llama_shaped_vocab())
    rng = np.random.default_rng(4)
    long_toks = ["".join(chr(c) for c in rng.integers(0x61, 0x64, size=L)) for L in (65, 70, 80, 150, 300) for _ in range(10)]
    for t in long_toks:
        t2i.setdefault(t, len(t2i))
    v = Vocab(t2i, 0)
    encl = Encoder(v)
    encl.debug_counter_bias(bias)
    long_ = ["x" + "".join(chr(c) for c in rng.integers(0x61, 0x64, size=rng.integers(65, 400))) for _ in range(200)]
    for k in range(100):
        a, b = long_toks[k % len(long_toks)], long_toks[(7 * k + 3) % len(long_toks)]
        long_.append("x" + a + "ab" + b[: (k * 13) % len(b)] + " " + b)
    text, offs = _csr(long_)
    got = encl.encode_csr(text, offs)
    ref = oracle.OracleVocab(t2i).encode_csr(text, offs)
    _cmp_csr(got, ref)
    assert np.array_equal(got[3], ref[3])
    # (3) the far-pair base: optimal predecessors more than 64 atoms back, listed by dpt_dp_host_far
    longs = ["".join(chr(c) for c in rng.integers(0x61, 0x64, size=L)) for L in (65, 66, 70, 80, 100, 150, 300)]
    u, w = longs[2], longs[3]
    fv = {"a", "b", "c", "x", "ab", "bc", "ca"} | set(longs) | {u + w[:3], w[3:], u[:-2], u[-2:] + w}
    words = [u + w, "x" + u + w, u + w + "ab", longs[0] + longs[1], longs[6] + "abc" + longs[5]]
    words += [longs[k % 7] + "abc"[: k % 4] + longs[(3 * k + 1) % 7][: 60 + k] for k in range(25)]
    ft2i = {t: i for i, t in enumerate(sorted(fv))}
    plain, biased = Encoder(Vocab(ft2i, 0)), Encoder(Vocab(ft2i, 0))
    biased.debug_counter_bias(bias)
    ftext, foffs, fcut = atoms_to_csr([list(wd) for wd in words])
    r0 = plain.dp(ftext, foffs, cut_mask=fcut, edges=True, far=True)
    r1 = biased.dp(ftext, foffs, cut_mask=fcut, edges=True, far=True)
    for x, y in zip(r0[:3], r1[:3]):
        assert np.array_equal(x, y)
    assert len(r0[3]) >= 5
    assert sorted(map(tuple, r0[3].tolist())) == sorted(map(tuple, r1[3].tolist()))


@pytest.mark.parametrize("n", [4095, 8192, 65535, 65536, 100003])
def test_work_partitions_vs_oracle(n, engines, oracles):
    """First-pass work distribution (tokenize_kernel: min(16, n / 4096) partition counters, claims of
    4 strings, a used-up mask): batch sizes at and around the partition-count steps, ragged strings
    (uneven work, so waves leave their first partition), three calls on one ctx (the counters and
    the mask are reset by the finish kernel's last block) -- every string exactly once, vs the oracle."""
    from dptok import synth
    rng = np.random.default_rng(n)
    text, offs = synth.random_ascii_corpus(n, 64, seed=n)
    cut = rng.integers(0, 65, size=n)
    cut[rng.random(n) < 0.02] = 0
    parts = [text[i * 64:i * 64 + int(cut[i])].tobytes() for i in range(n)]
    offs = np.zeros(n + 1, np.uint64)
    offs[1:] = np.cumsum([len(p) for p in parts])
    text = np.frombuffer(b"".join(parts) + b"\0", np.uint8)
    ref = oracles["llama32k"].encode_csr(text, offs)
    for _ in range(3):
        _cmp_csr(engines["llama32k"].encode_csr(text, offs), ref)


def test_encode_padded_matches_csr(vocabs, engines):
    """dpt_encode_padded (ids left at each string's byte offset, per-string counts, no finish pass)
    equals dpt_encode's CSR output on ragged strings -- empty ones, words over 256 bytes (the
    2048-byte pass) and over 2048 bytes (the unbounded pass, which writes into the caller's buffer) --
    over repeated calls on one ctx interleaved with dpt_encode (the counter resets of both paths)."""
    torch = pytest.importorskip("torch")
    from dptok import synth
    enc = engines["llama32k"]
    s = torch.cuda.current_stream().cuda_stream
    rng = np.random.default_rng(5)
    text, offs = synth.random_ascii_corpus(30000, 128, seed=51)
    parts = [text[i * 128:i * 128 + int(rng.integers(0, 129))].tobytes() for i in range(30000)]
    parts[7] = b"x" * 900                  # one word over 256 bytes
    parts[9] = b"ab" * 1500                # one word over 2048 bytes
    parts[11] = b""
    offs = np.zeros(len(parts) + 1, np.uint64)
    offs[1:] = np.cumsum([len(p) for p in parts])
    text = np.frombuffer(b"".join(parts) + b"\0", np.uint8)
    n, nb = len(parts), int(offs[-1])
    dt = torch.from_numpy(np.array(text)).cuda()
    do = torch.from_numpy(offs.view(np.int64)).cuda()
    for rep in range(3):
        ids = torch.full((nb,), -9, dtype=torch.int32, device="cuda")
        io = torch.empty(n + 1, dtype=torch.int64, device="cuda")
        st = torch.empty(n, dtype=torch.int32, device="cuda")
        enc.encode_device(dt.data_ptr(), nb, do.data_ptr(), n, ids.data_ptr(), nb, io.data_ptr(), st.data_ptr(), stream=s)
        pids = torch.full((nb,), -9, dtype=torch.int32, device="cuda")
        cnt = torch.full((n,), 7, dtype=torch.int64, device="cuda")
        pst = torch.empty(n, dtype=torch.int32, device="cuda")
        enc.encode_device_padded(dt.data_ptr(), nb, do.data_ptr(), n, pids.data_ptr(), nb, cnt.data_ptr(), pst.data_ptr(), stream=s)
        torch.cuda.synchronize()
        off_h = io.cpu().numpy().view(np.uint64)
        ids_h, pids_h, cnt_h = ids.cpu().numpy(), pids.cpu().numpy(), cnt.cpu().numpy()
        assert np.array_equal(pst.cpu().numpy(), st.cpu().numpy())
        assert np.array_equal(cnt_h.astype(np.uint64), np.diff(off_h)), rep
        for i in range(n):
            a, b = int(offs[i]), int(off_h[i])
            c = int(cnt_h[i])
            assert np.array_equal(pids_h[a:a + c], ids_h[b:b + c]), (rep, i)


def test_bloom_words_across_windows():
    """The 64-lane kernel's whole-word shortcut (a word that is ONE token is taken as such) relies on every
    256-byte window ending at a word start (window_bounds) and on the byte-stream walker never stepping past
    a word's end.  Strings of 240..900 bytes (2..4 windows) of BLOOM-scale words: tokens, tokens + 1..2
    letters (the prefix up to any cut is a token, the word is not), tokens less their last letter, short
    tokens -- every string against the oracle."""
    from bloom_fixture import big_vocab
    from dptok import Encoder, Vocab, synth
    from oracle import oracle
    t2i = big_vocab()
    longs, shorts = synth.bloom_word_pool(t2i)
    rng = np.random.default_rng(21)
    sp = synth.BYTE_SPACE
    parts, cuts = [], []
    for _ in range(3000):
        target, n, buf, cut = int(rng.integers(240, 900)), 0, bytearray(), bytearray()
        while n < target:
            r = rng.random()
            w = longs[int(rng.integers(len(longs)))]
            if 0.3 <= r < 0.6:
                w = w + "".join(rng.choice(list("xqz"), size=int(rng.integers(1, 3))))
            elif 0.6 <= r < 0.8:
                w = w[:-1]
            elif r >= 0.8:
                w = shorts[int(rng.integers(len(shorts)))]
            atoms = ([sp] if buf else []) + list(w)
            for k, a in enumerate(atoms):
                e = a.encode("utf-8")
                buf += e
                cut += bytes([3 if k == 0 else 2]) + b"\x00" * (len(e) - 1)
            n += len(w) + 2
        parts.append(bytes(buf))
        cuts.append(bytes(cut))
    offs = np.zeros(len(parts) + 1, dtype=np.uint64)
    offs[1:] = np.cumsum([len(p) for p in parts], dtype=np.uint64)
    text = np.frombuffer(b"".join(parts), dtype=np.uint8).copy()
    cut = np.frombuffer(b"".join(cuts), dtype=np.uint8).copy()
    got = Encoder(Vocab(t2i, 0)).encode_csr(text, offs, mode="atoms", cut_mask=cut)
    ref = oracle.OracleVocab(t2i).encode_csr(text, offs, mode=oracle.ATOMS, cut_mask=cut)
    _cmp_csr(got, ref)
    assert (got[2] == 0).sum() > 2500


def test_one_string_calls_vs_oracle(engines, oracles):
    """The drop-in's per-string call (reference main_analyze_s2orc.py:74-78: one dp_tokenize(str) per row) runs the
    one-string kernel -- lane-mode B and its C1 walks across the whole wave (SOLO) -- when the host's scan rules out
    the long-word passes: raw-mode strings of every corpus shape and llama-mode (PRESPLIT) ones, one call each,
    against the oracle (multi-window abstracts, Arabic, the golden edge cases, tie-heavy toy strings)."""
    from dptok import synth
    from oracle import oracle
    texts = synth.unpack(*synth.random_ascii_corpus(120, 256, seed=31))
    texts += synth.unpack(*synth.s2orc_like_corpus(40, seed=32))
    texts += synth.unpack(*synth.arabic_corpus(60, seed=33))
    texts += [c["text"] for c in load_golden("edge_llama32k.json.gz")["cases"] if not c.get("skipped")]
    for name in ("llama32k", "toy1k"):
        enc, ov = engines[name], oracles[name]
        for t in texts:
            got = enc.encode_strs([t])[0]
            rids, roff, rst, _ = ov.encode_csr(*_csr([t]))
            assert got == (rids[int(roff[0]):int(roff[1])].tolist(), int(rst[0])), (name, t[:60])
    # llama mode: one pre-split string per call (the '▁'-compressed windows included)
    text, offs = synth.random_ascii_corpus(60, 256, seed=34)
    t2, o2, cut = synth.llama_words(text, offs)
    enc, ov = engines["llama32k"], oracles["llama32k"]
    for i in range(60):
        a, b = int(o2[i]), int(o2[i + 1])
        one = np.array([0, b - a], dtype=np.uint64)
        got = enc.encode_csr(t2[a:b], one, mode="presplit", cut_mask=cut[a:b])
        ref = ov.encode_csr(t2[a:b], one, mode=oracle.PRESPLIT, cut_mask=cut[a:b])
        _cmp_csr(got, ref)


def test_mid_pass_words_257_to_512_bytes(engines, oracles):
    """The 512-byte pass (mid_kernel: PRESPLIT / ATOMS calls of 16-lane vocabularies) takes the strings whose word
    does not fit the first pass's 256-byte window: words of 200..530 bytes (its lane-mode B has chunks of up to 33
    boundaries), mixed with short ones, with and without '▁' markers, in PRESPLIT and ATOMS mode -- against the
    oracle; words over 512 bytes go on to the 2048-byte pass."""
    from dptok.engine import pack_word_atoms
    from oracle import oracle
    rng = np.random.default_rng(41)
    alpha = [chr(c) for c in range(0x21, 0x7F)]
    strings = []
    for k in range(600):
        words = []
        for _ in range(int(rng.integers(1, 4))):
            L = int(rng.integers(200, 531)) if rng.random() < 0.6 else int(rng.integers(1, 40))
            w = "".join(rng.choice(alpha, size=L))
            words.append(("▁" + w) if (words and k % 2) else w)
        strings.append(words)
    enc, ov = engines["llama32k"], oracles["llama32k"]
    # PRESPLIT: words as UTF-8 text + a word-start mask
    parts, cuts = [], []
    for words in strings:
        b = bytearray(); c = bytearray()
        for w in words:
            e = w.encode("utf-8")
            c += b"\x01" + b"\x00" * (len(e) - 1)
            b += e
        parts.append(bytes(b)); cuts.append(bytes(c))
    offs = np.zeros(len(parts) + 1, dtype=np.uint64)
    offs[1:] = np.cumsum([len(p) for p in parts], dtype=np.uint64)
    text = np.frombuffer(b"".join(parts), dtype=np.uint8).copy()
    cut = np.frombuffer(b"".join(cuts), dtype=np.uint8).copy()
    got = enc.encode_csr(text, offs, mode="presplit", cut_mask=cut)
    ref = ov.encode_csr(text, offs, mode=oracle.PRESPLIT, cut_mask=cut)
    _cmp_csr(got, ref)
    assert np.array_equal(got[3], ref[3])
    assert (got[2] == 0).sum() > 500
    # ATOMS: the same words, every code point an atom
    t2, o2, c2 = pack_word_atoms([[list(w) for w in words] for words in strings])
    got = enc.encode_csr(t2, o2, mode="atoms", cut_mask=c2)
    ref = ov.encode_csr(t2, o2, mode=oracle.ATOMS, cut_mask=c2)
    _cmp_csr(got, ref)
