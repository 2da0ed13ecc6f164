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
import os

HERE = os.path.dirname(os.path.abspath(__file__))
SNAPSHOT = "models--bigscience--bloom-3b/snapshots/52bc5b43010b4844513826b8be3f78c7344c37d7"


def make_hf_cache(root: str) -> str:
    d = os.path.join(root, SNAPSHOT)
    os.makedirs(d, exist_ok=True)
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
