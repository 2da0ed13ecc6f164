#!/usr/bin/env python3
"""Build the synthetic BLOOM-shaped tokenizer used by the row-f3 fixtures (TEST INFRASTRUCTURE).

``bigscience/bloom-3b`` is not available offline, so the BLOOM adapter
(reference packages/tokenizer_utils.py:98-181) is pinned with a small byte-level BPE trained
here with the `tokenizers` library: BLOOM's pre-tokenizer shape (a regex Split, isolated,
then ByteLevel without its own regex), the 256-character byte alphabet, a few special
tokens and ~1500 merges-derived tokens.  Merges are written in the "a b" string form of the
2022 BLOOM tokenizer.json (the form the reference's ``merge.split()`` parses).

Output: tests/golden/bloom_synth_tokenizer.json.gz  (deterministic for a given tokenizers
version; the committed file is what the tests use).

``--big``: the BLOOM-scale variant -- 250,680 entries like bloom-3b's
vocabulary, trained on a 23 MB synthetic corpus that repeats 4000 words of 17..40 letters, so
~14k tokens are longer than 16 code points (the one-string-per-wave `tokenize_kernel<256,64,..>`)
and most ids are past 32767 (int32 staging).  Output: tests/golden/bloom_big_tokenizer.json.xz
(~2 MB; training takes ~25 s).
"""
import gzip
import json
import lzma
import os
import random
import sys
import tempfile

from tokenizers import Regex, Tokenizer, decoders, models, pre_tokenizers, trainers

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "bloom_synth_tokenizer.json.gz")
OUT_BIG = os.path.join(HERE, "bloom_big_tokenizer.json.xz")
BIG_VOCAB = 250680
SPLIT = " ?[^(\\s|[.,!?…。，、।۔،])]+"


def corpus(n=4000, seed=3):
    rnd = random.Random(seed)
    letters = "etaoinshrdlucmfwypvbgkjqxz"
    arabic = [chr(c) for c in range(0x0621, 0x064B)]

    def word():
        r = rnd.random()
        if r < 0.8:
            return "".join(rnd.choice(letters) for _ in range(rnd.randint(1, 9)))
        if r < 0.9:
            return "".join(rnd.choice(arabic) for _ in range(rnd.randint(2, 6)))
        return str(rnd.randint(0, 9999))

    for _ in range(n):
        yield " ".join(word() for _ in range(rnd.randint(5, 25))) + rnd.choice([".", ",", "!", "?", "", "\n"])


def big_corpus(seed=5):
    """Sentences over three word pools: 4000 long words (17..40 letters), 400k ordinary words
    (2..12 letters, half of the draws Pareto-skewed towards the first ones), 30k Arabic words,
    and numbers."""
    rnd = random.Random(seed)
    letters = "etaoinshrdlucmfwypvbgkjqxz"
    arabic = [chr(c) for c in range(0x0621, 0x064B)]
    longw = ["".join(rnd.choice(letters) for _ in range(rnd.randint(17, 40))) for _ in range(4000)]
    words = ["".join(rnd.choice(letters) for _ in range(rnd.randint(2, 12))) for _ in range(400000)]
    ar_words = ["".join(rnd.choice(arabic) for _ in range(rnd.randint(2, 8))) for _ in range(30000)]
    lines = []
    for _ in range(200000):
        ws = []
        for _ in range(rnd.randint(5, 20)):
            r = rnd.random()
            if r < 0.08:
                ws.append(longw[int(rnd.paretovariate(1.0)) % len(longw)] if rnd.random() < 0.5 else rnd.choice(longw))
            elif r < 0.85:
                ws.append(words[min(int(rnd.paretovariate(0.6)) - 1, len(words) - 1)] if rnd.random() < 0.5
                          else rnd.choice(words))
            elif r < 0.95:
                ws.append(rnd.choice(ar_words))
            else:
                ws.append(str(rnd.randint(0, 99999)))
        lines.append(" ".join(ws) + rnd.choice([".", ",", "!", "?", "", "\n"]))
    return lines


def train(lines, vocab_size):
    tok = Tokenizer(models.BPE(unk_token=None))
    tok.pre_tokenizer = pre_tokenizers.Sequence([
        pre_tokenizers.Split(Regex(SPLIT), behavior="isolated"),
        pre_tokenizers.ByteLevel(add_prefix_space=False, use_regex=False)])
    tok.decoder = decoders.ByteLevel()
    trainer = trainers.BpeTrainer(vocab_size=vocab_size, initial_alphabet=pre_tokenizers.ByteLevel.alphabet(),
                                  special_tokens=["<unk>", "<s>", "</s>", "<pad>"], show_progress=False)
    tok.train_from_iterator(lines, trainer)
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "tokenizer.json")
        tok.save(p)
        with open(p) as fh:
            tj = json.load(fh)
    tj["model"]["merges"] = [m if isinstance(m, str) else " ".join(m) for m in tj["model"]["merges"]]
    return tj


def main_big():
    tj = train(big_corpus(), BIG_VOCAB)
    with lzma.open(OUT_BIG, "wb", preset=9) as fh:
        fh.write(json.dumps(tj, ensure_ascii=False, sort_keys=False).encode("utf-8"))
    v = tj["model"]["vocab"]
    print(OUT_BIG, len(v), "tokens,", len(tj["model"]["merges"]), "merges,",
          sum(len(t) > 16 for t in v), "longer than 16 code points")


def main():
    tok = Tokenizer(models.BPE(unk_token=None))
    tok.pre_tokenizer = pre_tokenizers.Sequence([
        pre_tokenizers.Split(Regex(SPLIT), behavior="isolated"),
        pre_tokenizers.ByteLevel(add_prefix_space=False, use_regex=False)])
    tok.decoder = decoders.ByteLevel()
    trainer = trainers.BpeTrainer(vocab_size=1800, initial_alphabet=pre_tokenizers.ByteLevel.alphabet(),
                                  special_tokens=["<unk>", "<s>", "</s>", "<pad>"], show_progress=False)
    tok.train_from_iterator(corpus(), trainer)
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "tokenizer.json")
        tok.save(p)
        with open(p) as fh:
            tj = json.load(fh)
    tj["model"]["merges"] = [m if isinstance(m, str) else " ".join(m) for m in tj["model"]["merges"]]
    with gzip.GzipFile(OUT, "wb", mtime=0) as fh:
        fh.write(json.dumps(tj, ensure_ascii=False, sort_keys=False).encode("utf-8"))
    print(OUT, len(tj["model"]["vocab"]), "tokens,", len(tj["model"]["merges"]), "merges")


if __name__ == "__main__":
    main_big() if sys.argv[1:] == ["--big"] else main()
