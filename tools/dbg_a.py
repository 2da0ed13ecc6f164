"""Debug: statuses/ids of a few strings through a given libdpt (DPT_LIB) vs the C oracle."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dp-tokenization_amd")]
import numpy as np
from dptok import Encoder, Vocab, synth, pack_strings
from oracle import oracle
texts = ["ab " * 200, "ab " * 10, "ab " * 86, "ab " * 85, "ab " * 87, "ab " * 100, "ab" + " ab" * 199, "ab " * 199 + "ab"]
for name, t2i in (("llama", synth.llama_shaped_vocab()), ("toy", synth.toy_vocab())):
    text, offs = pack_strings(texts)
    g = Encoder(Vocab(t2i, 0)).encode_csr(text, offs)
    r = oracle.OracleVocab(t2i).encode_csr(text, offs)
    for k in range(len(texts)):
        a = g[0][int(g[1][k]):int(g[1][k + 1])]
        b = r[0][int(r[1][k]):int(r[1][k + 1])]
        print(name, k, "st", g[2][k], r[2][k], "cap", g[3][k], r[3][k], "ids_eq", np.array_equal(a, b), len(a), len(b))
