"""Diagnostic: lane-mode B/C1 mismatches vs the C oracle (cfg2 golden texts + random corpora),
repeated runs for determinism, and the per-token diff of the first bad strings."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dp-tokenization_amd"), os.path.join(ROOT, "tests")]
import numpy as np
from dptok import Encoder, Vocab, synth, pack_strings
from oracle import oracle
from conftest import load_golden
t2i = synth.llama_shaped_vocab()
inv = {v: k for k, v in t2i.items()}
enc = Encoder(Vocab(t2i, 0))
orc = oracle.OracleVocab(t2i)
g = load_golden("cfg2_llama32k.json.gz")
texts = [c["text"] for c in g["cases"]]
def check(texts, label, show=2):
    text, offs = pack_strings(texts)
    a = enc.encode_csr(text, offs); r = orc.encode_csr(text, offs)
    bad = []
    for i in range(len(texts)):
        x = a[0][int(a[1][i]):int(a[1][i+1])].tolist(); y = r[0][int(r[1][i]):int(r[1][i+1])].tolist()
        if x != y or a[2][i] != r[2][i]:
            bad.append(i)
            if len(bad) <= show:
                k = next((k for k in range(min(len(x), len(y))) if x[k] != y[k]), None)
                print(label, "string", i, "len", len(texts[i]), "n", len(x), len(y), "first diff", k, "status", a[2][i], r[2][i])
                if k is not None:
                    print("   gpu:", [inv.get(t, t) for t in x[max(0, k-4):k+5]])
                    print("   ref:", [inv.get(t, t) for t in y[max(0, k-4):k+5]])
                    print("   text:", repr(texts[i]))
    print(label, "bad", len(bad), "of", len(texts), bad[:20])
    return bad
for rep in range(3):
    check(texts, "golden batch rep%d" % rep, show=2 if rep == 0 else 0)
b = check(texts[:8], "golden first 8")
for i in range(8):
    check([texts[i]], "single %d" % i, show=0)
tx, of = synth.random_ascii_corpus(4096, 256, seed=3)
check(synth.unpack(tx, of), "random 4096", show=1)
