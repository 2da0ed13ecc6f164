"""Debug: which batch compositions break "ab "*200 (DPT_LIB vs the C oracle)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dp-tokenization_amd")]
import numpy as np
from dptok import Encoder, Vocab, synth, pack_strings
from oracle import oracle
rng = np.random.default_rng(23)
pool = [chr(c) for c in range(0x20, 0x7F)] * 3 + ["\n", "\t", "\x01", "\x7f", "  ", " \n", "\n "]
rnd = []
for k in range(3000):
    n = int(rng.integers(0, 900)) if k % 4 else int(rng.integers(200, 320))
    rnd.append("".join(rng.choice(pool, size=n)))
tail = ["\n" * 300, " " * 300, "a" * 600, ("ab " * 200), "\t" * 257]
t2i = synth.llama_shaped_vocab()
enc, orc = Encoder(Vocab(t2i, 0)), oracle.OracleVocab(t2i)
cases = {"full": rnd + tail, "tail": tail, "sp+ab": [" " * 300, "ab " * 200], "ab*8": ["ab " * 200] * 8,
         "rnd+ab": rnd + ["ab " * 200], "sp300*3+ab": [" " * 300] * 3 + ["ab " * 200], "nl+sp+ab": ["\n" * 300, " " * 300, "ab " * 200],
         "sp20+ab": [" " * 20, "ab " * 200], "x+ab": ["xyz", "ab " * 200], "sp256+ab": [" " * 256, "ab " * 200],
         "ab+sp": ["ab " * 200, " " * 300]}
for name, texts in cases.items():
    text, offs = pack_strings(texts)
    g, r = enc.encode_csr(text, offs), orc.encode_csr(text, offs)
    bad = np.nonzero((g[2] != r[2]) | (g[3] != r[3]))[0]
    print(name, "bad", bad[:8].tolist(), [(int(g[2][k]), int(r[2][k]), int(g[3][k]), int(r[3][k])) for k in bad[:4]])
