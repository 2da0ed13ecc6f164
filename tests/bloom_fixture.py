"""TEST INFRASTRUCTURE: a BLOOM-shaped tokenizer object for the row-f3 adapter.

``bigscience/bloom-3b`` cannot be downloaded offline.  ``tests/golden/bloom_synth_tokenizer.json.gz``
(made by tests/golden/make_bloom_tokenizer.py) is a small byte-level BPE with BLOOM's
pre-tokenizer shape; this module lays it out where the reference reads it
(``{HF_CACHE_DIR}/models--bigscience--bloom-3b/snapshots/<sha>/tokenizer.json``,
reference packages/tokenizer_utils.py:111) and wraps it in ``transformers``'
``PreTrainedTokenizerFast`` -- the object type the reference's callers pass
(``_tokenizer.pre_tokenizer.pre_tokenize_str``, ``convert_ids_to_tokens``, ``decode``).
"""
import gzip
import json
import lzma
import os

HERE = os.path.dirname(os.path.abspath(__file__))
SNAPSHOT = "models--bigscience--bloom-3b/snapshots/52bc5b43010b4844513826b8be3f78c7344c37d7"


BIG = os.path.join(HERE, "golden", "bloom_big_tokenizer.json.xz")


def big_tokenizer_bytes() -> bytes:
    """tokenizer.json of the BLOOM-scale synthetic byte-level BPE (250,680 entries,
    tests/golden/make_bloom_tokenizer.py --big)."""
    with lzma.open(BIG, "rb") as fh:
        return fh.read()


def big_vocab() -> dict:
    """``{token: enumeration index}`` of the BLOOM-scale vocabulary -- the ``vocab_to_index`` of
    reference tokenizer_utils.py:104-108."""
    return {t: i for i, t in enumerate(json.loads(big_tokenizer_bytes())["model"]["vocab"])}


def make_hf_cache(root: str, big: bool = False) -> str:
    d = os.path.join(root, SNAPSHOT)
    os.makedirs(d, exist_ok=True)
    if big:
        data = big_tokenizer_bytes()
    else:
        with gzip.open(os.path.join(HERE, "golden", "bloom_synth_tokenizer.json.gz"), "rb") as fh:
            data = fh.read()
    with open(os.path.join(d, "tokenizer.json"), "wb") as fh:
        fh.write(data)
    return root


def bloom_tokenizer(hf_cache: str):
    from transformers import PreTrainedTokenizerFast
    return PreTrainedTokenizerFast(tokenizer_file=os.path.join(hf_cache, SNAPSHOT, "tokenizer.json"))


def bloom_texts(n: int = 300, seed: int = 17):
    """Sentences for the adapter fixtures: BPE-covered words, Arabic, digits, punctuation,
    accents, CJK, 4-byte emoji, runs of spaces, tabs, newlines, and the empty string."""
    import random
    rnd = random.Random(seed)
    letters = "etaoinshrdlucmfwypvbgkjqxz"
    extra = ["café", "naïve", "über", "中文字", "😀", "🤖x", "\t", "  ", "\n\n", "...", "?!", "1984", "-", "'s"]
    arabic = [chr(c) for c in range(0x0621, 0x064B)]
    out = ["", " ", "a", "hello world", " leading", "trailing ", "two  spaces", "line\nbreak"]
    while len(out) < n:
        ws = []
        for _ in range(rnd.randint(1, 18)):
            r = rnd.random()
            if r < 0.7:
                ws.append("".join(rnd.choice(letters) for _ in range(rnd.randint(1, 12))))
            elif r < 0.8:
                ws.append("".join(rnd.choice(arabic) for _ in range(rnd.randint(1, 7))))
            else:
                ws.append(rnd.choice(extra))
        out.append(" ".join(ws) + rnd.choice(["", ".", ",", "!", " ?"]))
    return out


def bloom_big_texts(vocab: dict, n: int = 400, seed: int = 29):
    """Sentences for the BLOOM-scale fixtures: the vocabulary's long tokens (> 16 code points) as
    words, glued in twos and threes (words of 40..120 atoms), cut short or extended by a few
    letters (the DP must split them), ordinary words, Arabic, digits, punctuation, accents and
    emoji, runs of spaces and newlines."""
    import random
    rnd = random.Random(seed)
    letters = "etaoinshrdlucmfwypvbgkjqxz"
    longs = sorted(t[1:] if t.startswith("\u0120") else t for t in vocab if len(t) > 16 and t.strip("\u0120").isalpha()
                   and t.strip("\u0120").isascii())
    arabic = [chr(c) for c in range(0x0621, 0x064B)]
    extra = ["café", "naïve", "über", "中文字", "😀", "🤖x", "\t", "  ", "\n\n", "...", "?!", "1984", "-", "'s"]
    out = ["", " ", "a", longs[0], " " + longs[1], longs[2] + longs[3], longs[4][:-1], longs[5] + "ing"]
    while len(out) < n:
        ws = []
        for _ in range(rnd.randint(1, 14)):
            r = rnd.random()
            if r < 0.25:
                ws.append(rnd.choice(longs))
            elif r < 0.35:
                ws.append("".join(rnd.choice(longs) for _ in range(rnd.randint(2, 3))))
            elif r < 0.45:
                w = rnd.choice(longs)
                ws.append(w[:rnd.randint(3, len(w) - 1)] + "".join(rnd.choice(letters) for _ in range(rnd.randint(0, 4))))
            elif r < 0.8:
                ws.append("".join(rnd.choice(letters) for _ in range(rnd.randint(1, 12))))
            elif r < 0.9:
                ws.append("".join(rnd.choice(arabic) for _ in range(rnd.randint(1, 7))))
            else:
                ws.append(rnd.choice(extra))
        out.append(" ".join(ws) + rnd.choice(["", ".", ",", "!", " ?"]))
    return out
