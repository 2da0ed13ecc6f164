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
        assert dp_tokenize(c["text"]) == c["ids"], c["text"]
    assert isinstance(decode(cs[30]["ids"]), str)
    eng = dp_tokenize.engine
    eng.profile(True)
    got = dp_tokenize.batch([c["text"] for c in cs])
    _, launches = eng.profile_read()
    eng.profile(False)
    assert launches == 1                                          # one pre-split launch for the batch
    bad = [c["text"] for c, g in zip(cs, got) if g != c["ids"]]
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
