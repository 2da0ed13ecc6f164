"""TEST INFRASTRUCTURE: a real SentencePiece Llama-style tokenizer for the llama-mode parity pin.

The reference's default pre-tokenizer (packages/tokenizer_utils.py:24-31, selected at :52 and used
by main_analyze_s2orc.py:74,256) runs ``tokenizer.encode`` of a Llama-2 ``LlamaTokenizer``.  No
Llama-2 ``tokenizer.model`` exists offline, so ``tests/golden/make_sp_llama.py``
trains one HERE with the installed ``sentencepiece`` 0.2.2 and the Llama-2 trainer settings
(BPE, 32000 pieces, byte_fallback, split_digits, add_dummy_prefix, no whitespace folding,
identity normaliser, pieces of <= 16 characters, <unk>/<s>/</s> = 0/1/2, bytes <0x00>..<0xFF> =
3..258) on synthetic text, and commits the model (``tests/golden/sp_llama32k.model``).

Two tokenizer objects over that one model, both with the interface the reference uses
(``get_vocab()``, ``encode(str)`` with BOS first, ``decode(ids)``):

* ``hf_llama(path)`` -- ``transformers.LlamaTokenizer`` (5.15, a ``tokenizers`` backend converted
  from the SentencePiece model) with ``add_bos_token=True`` as in Llama-2's tokenizer config;
* ``SPLlama(path)`` -- the SentencePiece processor itself plus BOS: what the slow
  ``LlamaTokenizer`` of older ``transformers`` returned from ``encode``.

They segment some inputs differently (leading and repeated spaces, literal ``<s>``), which is the
point of pinning both: the drop-in must reproduce the reference's composition for whatever the
tokenizer object returns.
"""
from __future__ import annotations

import os
import shutil
import tempfile
from typing import Dict, List

HERE = os.path.dirname(os.path.abspath(__file__))
MODEL = os.path.join(HERE, "golden", "sp_llama32k.model")


class SPLlama:
    """SentencePiece processor with Llama's BOS (the slow LlamaTokenizer's encode)."""

    def __init__(self, path: str = MODEL):
        import sentencepiece as spm
        self.sp = spm.SentencePieceProcessor(model_file=path)
        self._vocab = {self.sp.id_to_piece(i): i for i in range(self.sp.get_piece_size())}

    def get_vocab(self) -> Dict[str, int]:
        return dict(self._vocab)

    def encode(self, text: str) -> List[int]:
        return [self.sp.bos_id()] + list(self.sp.encode(text))

    def decode(self, ids: List[int]) -> str:
        return "<s> " + self.sp.decode([i for i in ids if i != self.sp.bos_id()])


def hf_llama(path: str = MODEL):
    """transformers.LlamaTokenizer over the same model (BOS added, as Llama-2's config sets)."""
    from transformers import LlamaTokenizer
    d = tempfile.mkdtemp(prefix="sp_llama_")
    try:
        shutil.copy(path, os.path.join(d, "tokenizer.model"))
        return LlamaTokenizer.from_pretrained(d, add_bos_token=True)
    finally:
        shutil.rmtree(d, ignore_errors=True)


def llama_texts(n_random: int = 520, seed: int = 7) -> List[str]:
    """>= 500 strings for the llama-mode pin: edge cases (empty, whitespace runs, newlines, tabs,
    literal <s> / </s> / <0xNN>, leading / trailing spaces) and random mixes of pseudo-English,
    digits, punctuation, accented Latin, Arabic, CJK and 4-byte code points (byte fallback)."""
    import random
    rng = random.Random(seed)
    edge = ["", " ", "  ", "\n", "\n\n", "\t", "x", " x", "x ", "a  b", "a   b", "ab\ncd", "ab\n\ncd", "\nab",
            "<s>", "</s>", "<unk>", "<s> hello", "a<s>b", "<0x0A>", "<0x41>", "a<0x41>b", "<0xC3><0x9F>",
            "hello world", "the weather", "€uro", "ü ß", "中文字", "😀 smile", "السلام عليكم", "ab\tc",
            " leading", "trailing ", "  both  ", "12345 6.78", "x\r\ny", " nbsp", "▁literal", "▁▁x",
            "OptimalLengthTokenization", "midafternoon", "é", "ﬁ ligature", "a" * 300, "ab " * 100]
    pools = [
        lambda: "".join(rng.choice("etaoinshrdlucmfwypvbgkjqxz") for _ in range(rng.randint(1, 12))),
        lambda: str(rng.randint(0, 10 ** rng.randint(1, 8))),
        lambda: rng.choice([".", ",", ";", ":", "(", ")", "%", "-", "!", "?", "'", '"', "<", ">", "/"]),
        lambda: "".join(rng.choice("éèüößñçàâêîôûëïœæ") for _ in range(rng.randint(1, 4))),
        lambda: "".join(chr(rng.randint(0x0621, 0x064A)) for _ in range(rng.randint(1, 6))),
        lambda: "".join(chr(rng.randint(0x4E00, 0x4FFF)) for _ in range(rng.randint(1, 3))),
        lambda: chr(rng.randint(0x1F600, 0x1F64F)),
        lambda: rng.choice(["<s>", "</s>", "<0x0A>", "<0x%02X>" % rng.randint(0, 255), "▁"]),
    ]
    weights = [60, 8, 10, 6, 6, 4, 2, 4]
    seps = [" "] * 20 + ["  ", "\n", "\n\n", "\t", "", " \n "]
    out = list(edge)
    while len(out) < len(edge) + n_random:
        parts = []
        for _ in range(rng.randint(1, 40)):
            parts.append(rng.choices(pools, weights)[0]())
            parts.append(rng.choice(seps))
        s = "".join(parts)
        if rng.random() < 0.2:
            s = " " + s
        out.append(s)
    return out
