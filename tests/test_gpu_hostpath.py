"""Small host-path calls (round 4): dpt_encode_host skips the 2048-byte and unbounded passes' launches
when its own scan of the text shows no string can need them (dpt_api.cpp no_fallback_needed), and
brings the counter block back inside its one device-to-host copy.  The scan must agree with the
kernels' routing exactly, so the cases sit on both sides of every limit -- words of 256 / 257 bytes
(raw and pre-split), word starts exactly 256 bytes apart, atoms of 4 / 5 bytes (malformed UTF-8),
leading continuation bytes -- each as its own small call, checked against the C oracle."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _cases():
    rng = np.random.default_rng(21)

    def rnd(n):
        return bytes(int(c) for c in rng.integers(0x21, 0x7F, size=n))
    cases = []
    for L in (255, 256, 257, 300):
        cases.append(rnd(L))                                   # one word of L bytes
        cases.append(rnd(100) + b" " + rnd(L - 1))             # a second word of L bytes (space included)
        cases.append(rnd(L) + b" " + rnd(10))
    cases.append(rnd(256) + b" yy")                            # a word start exactly 256 bytes in
    cases.append(rnd(200) + b" " + rnd(255) + b" " + rnd(255))
    cont = bytes([0x80])
    for k in (2, 3, 4, 5):                                     # atoms of a lead byte + k-1 continuations
        cases.append(b"ab " + bytes([0xF0]) + cont * (k - 1) + b" cd")
    cases.append(cont * 4 + b"x y")                            # leading continuation bytes (the first atom)
    cases.append(cont * 5 + b"x y")
    cases.append("é中😀 x".encode() * 10)
    return cases


def test_small_calls_at_the_fallback_limits(vocabs):
    from dptok import Encoder, Vocab, pack_strings
    from oracle import oracle
    t2i = vocabs["llama32k"]
    enc, orc = Encoder(Vocab(t2i, 0)), oracle.OracleVocab(t2i)
    for b in _cases():
        offs = np.array([0, len(b)], dtype=np.uint64)
        text = np.frombuffer(b + b"\0", dtype=np.uint8)
        got = enc.encode_csr(text, offs)
        ref = orc.encode_csr(text, offs)
        for g, r, what in zip(got, ref, ("ids", "offsets", "status", "capped")):
            assert np.array_equal(g, r), (what, b[:40], len(b))
    # and all of them in one call (bytes: malformed UTF-8 does not round-trip through str)
    blob = b"".join(_cases())
    lens = [len(b) for b in _cases()]
    offs = np.zeros(len(lens) + 1, dtype=np.uint64)
    offs[1:] = np.cumsum(lens)
    text = np.frombuffer(blob + b"\0", dtype=np.uint8)
    got, ref = enc.encode_csr(text, offs), orc.encode_csr(text, offs)
    for g, r in zip(got, ref):
        assert np.array_equal(g, r)


def test_presplit_small_calls(vocabs):
    """Pre-split words (llama mode's layout) of 256 / 257 bytes and more, one small call each."""
    from dptok import Encoder, Vocab
    from dptok.engine import pack_presplit_words
    from oracle import oracle
    t2i = vocabs["llama32k"]
    enc, orc = Encoder(Vocab(t2i, 0)), oracle.OracleVocab(t2i)
    rng = np.random.default_rng(5)
    for L in (200, 256, 257, 400, 3000):
        words = ["\u2581" + "".join(chr(int(c)) for c in rng.integers(0x61, 0x7B, size=L - 3)), "\u2581ab", "c"]
        text, offs, cut, _, _ = pack_presplit_words([words])
        got = enc.encode_csr(text, offs, mode="presplit", cut_mask=cut)
        ref = orc.encode_csr(text, offs, mode=oracle.PRESPLIT, cut_mask=cut)
        for g, r, what in zip(got, ref, ("ids", "offsets", "status", "capped")):
            assert np.array_equal(g, r), (what, L)


def test_one_string_calls(vocabs):
    """One-string host-path calls run the first pass alone (EncodeLaunch::solo: ids straight into the
    output, id_off and the counter reset by the lone wave): every mode, empty and untokenizable
    strings, the 64-lane kernel's vocabulary, interleaved with multi-string calls on the same context
    (a counter the lone wave failed to reset would show in the next call)."""
    from dptok import Encoder, Vocab, pack_strings
    from oracle import oracle
    rng = np.random.default_rng(8)
    t2i_long = dict(vocabs["llama32k"])
    for L in (17, 24, 40):
        for _ in range(10):
            tok = "".join(chr(c) for c in rng.integers(0x61, 0x65, size=L))
            t2i_long.setdefault(tok, len(t2i_long))
    pool = [chr(c) for c in range(0x21, 0x7F)] + ["é", "中", "😀", "\n", " ", "  "]
    texts = ["", " ", "a", "\n", "中文 😀", "abcd" * 40] + \
            ["".join(rng.choice(pool, size=int(rng.integers(1, 250)))) for _ in range(40)] + \
            ["".join(chr(c) for c in rng.integers(0x61, 0x65, size=200))]
    for name, t2i in (("llama32k", vocabs["llama32k"]), ("toy1k", vocabs["toy1k"]), ("long", t2i_long)):
        enc, orc = Encoder(Vocab(t2i, 0)), oracle.OracleVocab(t2i)
        for k, s in enumerate(texts):
            text, offs = pack_strings([s])
            got, ref = enc.encode_csr(text, offs), orc.encode_csr(text, offs)
            for g, r, what in zip(got, ref, ("ids", "offsets", "status", "capped")):
                assert np.array_equal(g, r), (name, k, what, s[:30])
            if k % 7 == 3:   # a multi-string call between one-string calls
                text, offs = pack_strings(texts[:k + 2])
                got, ref = enc.encode_csr(text, offs), orc.encode_csr(text, offs)
                for g, r in zip(got, ref):
                    assert np.array_equal(g, r), (name, k, "batch")
