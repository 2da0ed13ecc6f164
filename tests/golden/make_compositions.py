#!/usr/bin/env python3
"""Reference outputs of ``inspect_tokenizer.obtain_token_compositions`` (reference
inspect_tokenizer.py:17-42) over the synthetic BLOOM-style byte-level BPEs' own merges.

Runs here only (imports the reference read-only, with make_golden.py's stubs).  Cases:
  * the 1,800-entry BPE (tests/golden/bloom_synth_tokenizer.json.gz): every token of two or
    more code points, merges passed as the list tokenizer.json holds;
  * the 250,680-entry BPE (bloom_big_tokenizer.json.xz): 40 tokens per length bucket from 2 to
    41 code points plus strings that are not tokens, merges passed as a set (membership is all the
    function uses; the list's O(n) scans make 250k merges slow, not different).
Writes tests/golden/compositions.json.gz: token, merge source ("small" / "big"), the
reference's list of decompositions (data only).
"""
from __future__ import annotations

import gzip
import json
import lzma
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import make_golden  # noqa: E402,F401  (stubs; the reference read-only)
import inspect_tokenizer  # noqa: E402

assert inspect_tokenizer.__file__.startswith("/root/reference"), inspect_tokenizer.__file__


def _merges(m):
    return [x if isinstance(x, str) else " ".join(x) for x in m]


def main():
    otc = inspect_tokenizer.obtain_token_compositions
    small = json.load(gzip.open(os.path.join(HERE, "bloom_synth_tokenizer.json.gz"), "rt", encoding="utf-8"))
    sv, sm = small["model"]["vocab"], _merges(small["model"]["merges"])
    cases = []
    for t in sv:
        if len(t) >= 2:
            cases.append({"token": t, "source": "small", "compositions": otc(t, sv, sm)})
    with lzma.open(os.path.join(HERE, "bloom_big_tokenizer.json.xz"), "rt", encoding="utf-8") as fh:
        big = json.load(fh)
    bv, bm = big["model"]["vocab"], set(_merges(big["model"]["merges"]))
    rng = random.Random(31)
    by_len = {}
    for t in bv:
        by_len.setdefault(len(t), []).append(t)
    picks = []
    for L in sorted(by_len):
        if L >= 2:
            picks += rng.sample(by_len[L], min(40, len(by_len[L])))
    # not tokens: a token plus a letter, two tokens glued
    picks += [rng.choice(picks) + "e" for _ in range(20)] + [rng.choice(picks) + rng.choice(picks) for _ in range(20)]
    for t in picks:
        cases.append({"token": t, "source": "big", "compositions": otc(t, bv, bm)})
    out = {"source": "reference inspect_tokenizer.obtain_token_compositions (inspect_tokenizer.py:17-42) over the "
                     "synthetic byte-level BPEs' merges", "cases": cases}
    path = os.path.join(HERE, "compositions.json.gz")
    with gzip.GzipFile(path, "wb", mtime=0) as f:
        f.write(json.dumps(out, ensure_ascii=False).encode("utf-8"))
    print(path, len(cases), "cases;", sum(len(c["compositions"]) for c in cases), "decompositions; max",
          max(len(c["compositions"]) for c in cases))


if __name__ == "__main__":
    main()
