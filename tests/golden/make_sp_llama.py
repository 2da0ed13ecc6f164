#!/usr/bin/env python3
"""Llama-mode golden vectors against REAL SentencePiece (run here, where /root/reference exists).

1. ``train``: trains ``tests/golden/sp_llama32k.model`` with sentencepiece 0.2.2 and the Llama-2
   trainer settings (see tests/sp_llama.py) on synthetic text (dptok.synth pseudo-English plus
   digits, accented Latin, Arabic; characters outside 99.95 % coverage fall back to <0xNN>).
2. ``cases``: for every text of ``sp_llama.llama_texts()`` and both tokenizer objects over that
   model (``transformers.LlamaTokenizer`` and the raw SentencePiece processor + BOS), runs the
   REFERENCE's own llama-mode composition -- ``pretokenize_with_llama(tokenizer, bidict(t2i))``
   (packages/tokenizer_utils.py:24-31, with its ``merge_tokens`` :7-22), then per word
   ``compute_shortest_tokenizations(word, vocab, False, None)`` + ``obtain_longest_token`` and
   ``t2i`` (:66-80 with the evident 4-argument call) -- imported read-only from /root/reference
   with the stubs of make_golden.py.  Writes tests/golden/sp_llama_cases.json.gz: text, the
   tokenizer's ids, the merged words, the reference's ids / status (data only).

Usage: python tests/golden/make_sp_llama.py [train] [cases] [decode]
"""
from __future__ import annotations

import gzip
import hashlib
import io
import json
import multiprocessing as mp
import os
import random
import signal
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(REPO, "dp-tokenization_amd"), os.path.join(REPO, "tests")]

from sp_llama import MODEL, SPLlama, hf_llama, llama_texts  # noqa: E402


def train():
    import sentencepiece as spm
    from dptok import synth
    text, offs = synth.s2orc_like_corpus(3000, seed=101)
    lines = []
    for s in synth.unpack(text, offs):
        lines.extend(s.split("\n"))
    rng = random.Random(5)
    extra = "é€üößñçàèìòùâêîôûäëïö"
    ar = [chr(c) for c in range(0x0621, 0x064B)]
    for _ in range(4000):
        w = []
        for _ in range(rng.randint(3, 20)):
            r = rng.random()
            if r < 0.05:
                w.append("".join(rng.choice(ar) for _ in range(rng.randint(2, 6))))
            elif r < 0.15:
                w.append(str(rng.randint(0, 100000)))
            else:
                w.append("".join(rng.choice("etaoinshrdlucmfwypvbgkjqxz" + extra[:rng.randint(0, 3)])
                                 for _ in range(rng.randint(1, 9))))
        lines.append(" ".join(w))
    m = io.BytesIO()
    spm.SentencePieceTrainer.train(
        sentence_iterator=iter(lines), model_writer=m, model_type="bpe", vocab_size=32000, byte_fallback=True,
        split_digits=True, add_dummy_prefix=True, remove_extra_whitespaces=False, normalization_rule_name="identity",
        allow_whitespace_only_pieces=True, max_sentencepiece_length=16, unk_id=0, bos_id=1, eos_id=2, pad_id=-1,
        character_coverage=0.9995, num_threads=1, minloglevel=2)
    with open(MODEL, "wb") as f:
        f.write(m.getvalue())
    print("model:", MODEL, len(m.getvalue()), "bytes")


_G = {}


def _init():
    sys.path.insert(0, HERE)
    import make_golden  # noqa: F401  (installs the stubs and imports the reference read-only)
    from packages.dp_tokenize import compute_shortest_tokenizations, obtain_longest_token
    from packages.tokenizer_utils import pretokenize_with_llama
    import packages
    assert packages.__file__.startswith("/root/reference"), packages.__file__   # the reference, not the drop-in
    _G["cst"], _G["olt"] = compute_shortest_tokenizations, obtain_longest_token
    _G["tok"] = {"hf": hf_llama(), "sp": SPLlama()}
    bidict = sys.modules["bidict"].bidict
    _G["t2i"] = {k: dict(t.get_vocab()) for k, t in _G["tok"].items()}
    _G["pre"] = {k: pretokenize_with_llama(t, bidict(_G["t2i"][k])) for k, t in _G["tok"].items()}

    def _alarm(signum, frame):
        raise TimeoutError()
    signal.signal(signal.SIGALRM, _alarm)


def _case(args):
    kind, text = args
    t2i = _G["t2i"][kind]
    vocab = set(t2i)
    signal.alarm(60)
    try:
        tok_ids = list(_G["tok"][kind].encode(text))
        words = _G["pre"][kind](text)
        ids, status = [], 0
        for w in words:
            try:
                toks, _ = _G["cst"](w, vocab, False, None)
            except IndexError:
                status = 2
                break
            if not toks:
                status = 1
                break
            ids.extend(t2i[x] for x in _G["olt"](toks))
        return {"tokenizer": kind, "text": text, "tok_ids": tok_ids, "words": words,
                "ids": ids if status == 0 else [], "status": status}
    except TimeoutError:
        return {"tokenizer": kind, "text": text, "skipped": True}
    finally:
        signal.alarm(0)


def cases():
    texts = llama_texts()
    jobs = [(k, t) for k in ("hf", "sp") for t in texts]
    with mp.Pool(8, initializer=_init) as pool:
        rows = pool.map(_case, jobs, chunksize=4)
    with open(MODEL, "rb") as f:
        sha = hashlib.sha256(f.read()).hexdigest()
    out = {"source": "reference pretokenize_with_llama + compute_shortest_tokenizations + obtain_longest_token "
                     "(packages/tokenizer_utils.py:24-31,66-80), real SentencePiece model trained here",
           "model_sha256": sha, "cases": rows}
    path = os.path.join(HERE, "sp_llama_cases.json.gz")
    with gzip.GzipFile(path, "wb", mtime=0) as f:
        f.write(json.dumps(out, ensure_ascii=False).encode("utf-8"))
    st = {}
    for r in rows:
        k = "skipped" if r.get("skipped") else r["status"]
        st[k] = st.get(k, 0) + 1
    print(path, len(rows), "cases, statuses", st)


def decode():
    """Adds to every case the reference's own ``decode_dp_tokenization(ids)`` (the second closure of
    ``dp_tokenize_llama``, packages/tokenizer_utils.py:82-84: ``llama_tokenizer.decode(ids)[4:]``),
    over the recorded ids -- the round-trip surface of main_analyze_s2orc.py:84-87."""
    sys.path.insert(0, HERE)
    import make_golden  # noqa: F401  (stubs; the reference read-only)
    from packages.tokenizer_utils import dp_tokenize_llama
    import packages
    assert packages.__file__.startswith("/root/reference"), packages.__file__
    toks = {"hf": hf_llama(), "sp": SPLlama()}
    dec = {k: dp_tokenize_llama(t, "llama")[1] for k, t in toks.items()}
    path = os.path.join(HERE, "sp_llama_cases.json.gz")
    with gzip.open(path, "rt", encoding="utf-8") as f:
        out = json.load(f)
    n = 0
    for c in out["cases"]:
        if c.get("skipped") or c["status"] != 0:
            continue
        c["decoded"] = dec[c["tokenizer"]](c["ids"])
        n += 1
    out["decode_source"] = "reference dp_tokenize_llama(tokenizer)[1] (packages/tokenizer_utils.py:82-84) over the ids"
    with gzip.GzipFile(path, "wb", mtime=0) as f:
        f.write(json.dumps(out, ensure_ascii=False).encode("utf-8"))
    print(path, "decoded", n, "cases")


if __name__ == "__main__":
    steps = sys.argv[1:] or ["train", "cases", "decode"]
    if "train" in steps:
        train()
    if "cases" in steps:
        cases()
    if "decode" in steps:
        decode()
