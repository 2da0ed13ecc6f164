"""CPU: dptok.synth.llama_words -- the pre-split form of bench.py's cfg2p / cfg4p workloads (llama mode) --
equals merge_tokens over the pieces of a real SentencePiece model (tests/golden/sp_llama32k.model, Llama-2
trainer settings) on text its pieces cover without byte fallback (reference tokenizer_utils.py:7-31)."""
import numpy as np
import pytest


def _words(text, offs, cut, i):
    b = bytes(text[int(offs[i]):int(offs[i + 1])])
    c = cut[int(offs[i]):int(offs[i + 1])]
    starts = [k for k in range(len(b)) if c[k]] + [len(b)]
    return [b[starts[j]:starts[j + 1]].decode("utf-8") for j in range(len(starts) - 1)]


def test_llama_words_match_sentencepiece_words():
    pytest.importorskip("sentencepiece")
    from sp_llama import hf_llama
    from dptok import pack_strings, synth
    from packages.tokenizer_utils import merge_tokens
    tok = hf_llama()
    inv = {v: k for k, v in tok.get_vocab().items()}
    rng = np.random.default_rng(3)
    texts = ["hello world", "a  b", "ab\ncd e", "z", "the weather is fine\ntoday"]
    for _ in range(200):
        words = ["".join(rng.choice(list("etaoinshrdlucmfwypvbgk"), size=int(rng.integers(1, 12)))) for _ in range(int(rng.integers(1, 30)))]
        seps = rng.choice([" ", " ", " ", " ", "  ", "\n"], size=len(words))
        texts.append("".join(w + (s if k + 1 < len(words) else "") for k, (w, s) in enumerate(zip(words, seps))))
    text, offs = pack_strings(texts)
    t2, o2, cut = synth.llama_words(np.asarray(text), offs)
    assert int(o2[-1]) == len(t2) == len(cut)
    for i, t in enumerate(texts):
        assert _words(t2, o2, cut, i) == merge_tokens([inv[x] for x in tok.encode(t)], sep="▁"), t


def test_llama_words_offsets_and_prefix():
    from dptok import synth
    text, offs = synth.random_ascii_corpus(64, 256, seed=9)
    t2, o2, cut = synth.llama_words(text, offs)
    for i in range(64):
        s = bytes(text[int(offs[i]):int(offs[i + 1])])
        p = bytes(t2[int(o2[i]):int(o2[i + 1])])
        assert p == "<s>▁".encode() + s.replace(b" ", "▁".encode())
        assert cut[int(o2[i])] == 1 and cut[int(o2[i]) + 3] == 1
        assert int(cut[int(o2[i]):int(o2[i + 1])].sum()) == 2 + s.count(b" ")
