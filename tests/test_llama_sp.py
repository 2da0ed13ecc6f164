"""Llama mode (the factory's default option) pinned against REAL SentencePiece.

tests/golden/sp_llama_cases.json.gz holds, for 565 texts and two tokenizer objects over the
SentencePiece model trained by tests/golden/make_sp_llama.py (transformers.LlamaTokenizer and the
raw SentencePiece processor + BOS), the reference's own llama-mode output:
pretokenize_with_llama + merge_tokens (packages/tokenizer_utils.py:7-31) then the per-word DP
and longest-token selection (:66-80).  Byte-fallback pieces (literal '<0xNN>' strings inside
words), the BOS word '<s>', '▁'-only pieces of whitespace runs, newlines and tabs all occur.

CPU: the tokenizer objects reproduce the recorded SentencePiece ids and the drop-in's host-side
merge gives the recorded words.  GPU: ``dp_tokenize_llama(tokenizer)`` is bit-exact per call and
in ONE launch for the whole batch.
"""
import hashlib

import pytest

from conftest import load_golden


@pytest.fixture(scope="module")
def sp_cases():
    from sp_llama import MODEL
    g = load_golden("sp_llama_cases.json.gz")
    with open(MODEL, "rb") as f:
        assert hashlib.sha256(f.read()).hexdigest() == g["model_sha256"]
    return g


@pytest.fixture(scope="module")
def tokenizers_():
    from sp_llama import SPLlama, hf_llama
    return {"hf": hf_llama(), "sp": SPLlama()}


def _by_kind(g, kind):
    return [c for c in g["cases"] if c["tokenizer"] == kind and not c.get("skipped")]


def test_fixture_coverage(sp_cases):
    for kind in ("hf", "sp"):
        cs = _by_kind(sp_cases, kind)
        assert len(cs) >= 500
        assert all(isinstance(c["decoded"], str) for c in cs)    # reference decode outputs (make_sp_llama.py decode)
        words = [w for c in cs for w in c["words"]]
        assert any("<0x" in w for w in words)                      # byte-fallback pieces
        assert any(w.strip("▁") == "" for w in words)             # '▁'-only pieces (whitespace runs)
        assert any("<0x0A>" in w for w in words)                   # newlines
        assert all(c["words"][0].startswith("<s>") for c in cs)   # BOS word first
        assert any(any(ord(ch) > 0x7F and ch != "▁" for ch in w) for w in words)   # non-ASCII atoms


@pytest.mark.parametrize("kind", ["hf", "sp"])
def test_host_pretokenization_matches_reference(kind, sp_cases, tokenizers_):
    """SentencePiece here segments like it did when the fixture was made, and the drop-in's
    pretokenize_with_llama merges the pieces into the reference's words."""
    from packages.tokenizer_utils import _InverseDict, pretokenize_with_llama
    tok = tokenizers_[kind]
    pre = pretokenize_with_llama(tok, _InverseDict(tok.get_vocab()))
    for c in _by_kind(sp_cases, kind):
        assert list(tok.encode(c["text"])) == c["tok_ids"], c["text"]
        assert pre(c["text"]) == c["words"], c["text"]


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["hf", "sp"])
def test_dp_tokenize_llama_real_sentencepiece(kind, sp_cases, tokenizers_):
    from packages.tokenizer_utils import dp_tokenize_llama
    dp_tokenize, decode = dp_tokenize_llama(tokenizers_[kind])   # default pretokenize_option='llama'
    cs = _by_kind(sp_cases, kind)
    for c in cs[:120]:                                            # the unchanged callers' per-string call
        ids = dp_tokenize(c["text"])
        assert ids == c["ids"], c["text"]
        # the round trip of main_analyze_s2orc.py:84-87: the reference's own decode output
        assert decode(ids) == c["decoded"], c["text"]
    eng = dp_tokenize.engine
    eng.profile(True)
    got = dp_tokenize.batch([c["text"] for c in cs] * 4)          # >= 2048 strings: the worker pool's path
    _, launches = eng.profile_read()
    eng.profile(False)
    assert launches == 1                                          # one pre-split launch for the batch
    assert dp_tokenize.host_pool._workers or dp_tokenize.host_pool._broken
    bad = [c["text"] for c, g in zip(cs * 4, got) if g != c["ids"]]
    assert not bad, bad[:3]


@pytest.mark.gpu
def test_encode_presplit_empty_word_order():
    """An empty word raises IndexError in the reference's loop unless an earlier word already
    failed (ValueError); strings without words produce no ids."""
    from dptok import Encoder, Vocab, STATUS_EMPTY_WORD, STATUS_NO_TOKENIZATION, STATUS_OK
    enc = Encoder(Vocab({"a": 0, "b": 1, "ab": 2, "▁a": 3}, 0))
    res = enc.encode_presplit([["ab", "", "a"], ["zz", "", "a"], [], ["a"], ["", "a"], ["a", "b", "ab"]])
    assert res[0] == ([], STATUS_EMPTY_WORD)
    assert res[1] == ([], STATUS_NO_TOKENIZATION)
    assert res[2] == ([], STATUS_OK)
    assert res[3] == ([0], STATUS_OK)
    assert res[4] == ([], STATUS_EMPTY_WORD)
    assert res[5] == ([0, 1, 2], STATUS_OK)


@pytest.mark.parametrize("kind", ["hf", "sp"])
def test_batched_host_pretokenization_equals_per_string(kind, sp_cases, tokenizers_):
    """The drop-in's batched llama-mode host side (packages/tokenizer_utils.batch_encoder + the
    array-gather PieceTable) gives, for every fixture text and a random ASCII / S2ORC-shaped sample,
    the ids of per-string ``tokenizer.encode`` and the exact pre-split buffers the word lists of
    ``pretokenize_with_llama`` + ``merge_tokens`` (reference tokenizer_utils.py:7-31) pack into."""
    import numpy as np
    from dptok import synth
    from dptok.engine import PieceTable, pack_presplit_words
    from packages.tokenizer_utils import _InverseDict, batch_encoder, pretokenize_with_llama
    tok = tokenizers_[kind]
    t2i = dict(tok.get_vocab())
    texts = [c["text"] for c in _by_kind(sp_cases, kind)]
    texts += synth.unpack(*synth.random_ascii_corpus(300, 256, seed=11))
    texts += synth.unpack(*synth.s2orc_like_corpus(30, seed=12))
    ids = batch_encoder(tok)(texts)
    assert ids == [list(tok.encode(t)) for t in texts]
    table = PieceTable(t2i)
    assert table.ok and not table.empty_piece
    text, offs, cut, cnt = table.pack(ids)
    pre = pretokenize_with_llama(tok, _InverseDict(t2i))
    words = [pre(t) for t in texts]
    t2, o2, c2, nw, cut_at = pack_presplit_words(words)
    assert all(k < 0 for k in cut_at)                   # no empty words
    assert np.array_equal(offs, o2) and np.array_equal(text, t2) and np.array_equal(cut, c2)
    assert np.array_equal(cnt > 0, np.asarray(nw) > 0)
    with pytest.raises(KeyError):
        table.pack([[1, 2], [len(table.present) + 5]])   # reference: vocab_bidict.inverse[token]


@pytest.mark.parametrize("kind", ["hf", "sp"])
def test_pretokenize_pool_equals_in_process(kind, tokenizers_):
    """dptok.hostpool.PretokenizePool (worker processes, python -m dptok._pretok_worker) returns the
    in-process buffers for a batch split into chunks, in order."""
    import numpy as np
    from dptok import synth
    from dptok.engine import PieceTable
    from dptok.hostpool import PretokenizePool
    from packages.tokenizer_utils import batch_encoder
    tok = tokenizers_[kind]
    texts = synth.unpack(*synth.random_ascii_corpus(1500, 128, seed=13)) + ["", " ", "a\nb"] * 20
    table, enc = PieceTable(dict(tok.get_vocab())), batch_encoder(tok)
    ref = table.pack(enc(texts))
    pool = PretokenizePool(tok, table, enc, procs=2, min_batch=1)
    try:
        got = pool.pack(texts)
        assert pool._workers and not pool._broken          # the workers ran it
        assert all(np.array_equal(a, b) for a, b in zip(got, ref))
    finally:
        pool.close()


def test_batch_encoder_falls_back_on_private_api_change(tokenizers_, monkeypatch):
    """the tokenizers fast path calls private transformers APIs; if their signature changes,
    the batch encoder switches to the public per-text encode instead of raising."""
    from packages.tokenizer_utils import batch_encoder
    tok = tokenizers_["hf"]
    texts = ["hello world", " a\nb", "", "OptimalLengthTokenization"]
    ref = [tok.encode(t) for t in texts]
    enc = batch_encoder(tok)

    class Backend:   # the Rust backend, with a changed batch signature
        def __init__(self, t):
            object.__setattr__(self, "_t", t)

        def __getattr__(self, k):
            return getattr(self._t, k)

        def __setattr__(self, k, v):
            setattr(self._t, k, v)

        def encode_batch_fast(self, *a, **k):
            raise TypeError("unexpected keyword argument")
    monkeypatch.setattr(tok, "_tokenizer", Backend(tok._tokenizer))
    assert enc(texts) == ref
    assert enc(texts) == ref   # (permanently per text now)


def test_worker_recv_times_out():
    """a pre-tokenization worker that never answers counts as a dead one (bounded wait)."""
    import os
    import time
    from dptok.hostpool import recv_msg
    r, w = os.pipe()
    try:
        f = os.fdopen(r, "rb", buffering=0)
        t0 = time.monotonic()
        with pytest.raises(TimeoutError):
            recv_msg(f, 0.3)
        assert time.monotonic() - t0 < 5
    finally:
        os.close(w)
        f.close()


def test_one_pool_per_tokenizer(tokenizers_):
    """adapters over the same tokenizer share one worker pool."""
    from dptok.engine import PieceTable
    from dptok.hostpool import shared_pool
    from packages.tokenizer_utils import batch_encoder
    tok = tokenizers_["sp"]
    table, enc = PieceTable(dict(tok.get_vocab())), batch_encoder(tok)
    assert shared_pool(tok, table, enc) is shared_pool(tok, table, enc)
