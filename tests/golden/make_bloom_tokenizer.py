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
"""
import gzip
import json
import os
import random
import tempfile

from tokenizers import Regex, Tokenizer, decoders, models, pre_tokenizers, trainers

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "bloom_synth_tokenizer.json.gz")
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
    main()
