"""The chunk algorithm of the lane-mode phases B and C1 (tokenize_kernel, G = 16, capless
windows), restated on the CPU by tools/lane_model.py, against the C oracle's selection on
tie-heavy vocabularies with long words (many chunks per word).  CPU only: this pins the design
the kernel implements; tests/test_gpu_parity.py::test_tie_heavy_long_words_vs_oracle checks
the kernel itself on the same generator."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))


def tie_heavy_case(rng, max_len=200, alphabet="abc"):
    """A capless vocabulary (every letter and '▁'+letter) with many short multi-letter tokens,
    and a text of long words over the same letters."""
    vocab = set(alphabet) | {"▁" + c for c in alphabet} | {"▁"}
    for _ in range(int(rng.integers(5, 40))):
        L = int(rng.integers(2, 6))
        t = "".join(rng.choice(list(alphabet), size=L))
        vocab.add(("▁" + t[1:]) if rng.random() < 0.2 else t)
    n = int(rng.integers(1, max_len))
    chars = rng.choice(list(alphabet) + [" "], size=n, p=[0.32, 0.32, 0.32, 0.04])
    text = alphabet[0] + "".join(chars)
    return sorted(vocab), text


@pytest.mark.parametrize("seed", range(4))
def test_lane_model_matches_oracle(seed):
    import lane_model
    from oracle import oracle
    from dptok import pack_strings
    rng = np.random.default_rng(100 + seed)
    for n in range(150):
        vocab, text = tie_heavy_case(rng, max_len=256 if n % 2 else 120)
        t2i = {t: i for i, t in enumerate(vocab)}
        txt, offs = pack_strings([text])
        ids, off, st, _ = oracle.OracleVocab(t2i).encode_csr(txt, offs)
        if st[0] != 0:
            continue
        want = [vocab[i] for i in ids.tolist()]
        assert lane_model.model(text, set(vocab)) == want, (text, vocab)


def test_lane_model_matches_reference_port_short():
    """Short words against the enumerate-then-select restatement of the reference itself."""
    import lane_model
    rng = np.random.default_rng(7)
    for _ in range(150):
        vocab, text = tie_heavy_case(rng, max_len=28)
        try:
            want = lane_model.ref_tokens(text, set(vocab))
        except ValueError:
            continue
        assert lane_model.model(text, set(vocab)) == want, (text, vocab)


@pytest.mark.parametrize("seed", range(4))
def test_lane_model64_matches_oracle(seed):
    """forward_lanes64 (the 64-lane kernel's capless B): tokens up to 40 letters, words up to 256."""
    import lane_model
    from oracle import oracle
    from dptok import pack_strings
    rng = np.random.default_rng(300 + seed)
    for n in range(120):
        vocab, text = tie_heavy_case(rng, max_len=256 if n % 2 else 120)
        vocab = set(vocab)
        for _ in range(int(rng.integers(0, 30))):   # long tokens: substrings of the text's words
            w = rng.choice(text.split(" "))
            if len(w) > 17:
                a = int(rng.integers(0, len(w) - 17)); b = a + int(rng.integers(17, min(40, len(w) - a) + 1))
                vocab.add(w[a:b])
        vocab = sorted(vocab)
        t2i = {t: i for i, t in enumerate(vocab)}
        txt, offs = pack_strings([text])
        ids, off, st, _ = oracle.OracleVocab(t2i).encode_csr(txt, offs)
        if st[0] != 0:
            continue
        want = [vocab[i] for i in ids.tolist()]
        assert lane_model.model64(text, set(vocab)) == want, (text, vocab)
