"""TEST INFRASTRUCTURE: a stand-in for ``AutoTokenizer.from_pretrained("meta-llama/Llama-2-7b-hf")``
(unavailable offline, SURVEY.md §0 finding 6) with the interface the reference uses:
``get_vocab()``, ``encode(str) -> List[int]`` (BOS first) and ``decode(List[int]) -> str``.

``encode`` imitates SentencePiece with byte fallback closely enough to exercise the llama-mode
pre-tokenization path (reference tokenizer_utils.py:24-31): a leading '▁', spaces -> '▁',
greedy longest-match pieces over the vocabulary, unknown characters as ``<0xNN>`` byte pieces.
It is NOT the real Llama-2 segmentation; parity for llama mode is pinned against the
reference's own composition run with this same object (tests/golden/make_golden.py).
"""
from __future__ import annotations

from typing import Dict, List


class FakeLlamaTokenizer:
    def __init__(self, t2i: Dict[str, int], max_piece: int = 16):
        self._t2i = dict(t2i)
        self._i2t = {v: k for k, v in self._t2i.items()}
        self._max = max_piece

    def get_vocab(self) -> Dict[str, int]:
        return dict(self._t2i)

    def encode(self, text: str) -> List[int]:
        s = "▁" + text.replace(" ", "▁")
        ids = [self._t2i["<s>"]]
        i = 0
        while i < len(s):
            for L in range(min(self._max, len(s) - i), 0, -1):
                piece = s[i:i + L]
                if piece in self._t2i:
                    ids.append(self._t2i[piece])
                    i += L
                    break
            else:
                for b in s[i].encode("utf-8"):
                    ids.append(self._t2i["<0x%02X>" % b])
                i += 1
        return ids

    def decode(self, ids: List[int]) -> str:
        out = []
        pend = bytearray()
        for t in ids:
            p = self._i2t[t]
            if len(p) == 6 and p.startswith("<0x") and p.endswith(">"):
                pend.append(int(p[3:5], 16))
                continue
            if pend:
                out.append(pend.decode("utf-8", "replace"))
                pend = bytearray()
            out.append(p)
        if pend:
            out.append(pend.decode("utf-8", "replace"))
        s = "".join(out).replace("▁", " ")
        if s.startswith("<s>"):
            s = "<s> " + s[3:].lstrip(" ")  # the "<s> " prefix the reference slices off ([4:])
        return s
