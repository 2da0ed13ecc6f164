"""CPU count (no GPU): dependent trie loads per phase-A walk on the BLOOM-scale corpus, one-byte steps
(the byte-stream walker, dpt_kernels.hip) against a two-byte step table -- (node, next two bytes) -> the node
after them + the terminal flag of the node between.

    python tools/pair_step_count.py [n_strings]       (default 20000)

A walk from atom j: the root table for the first two bytes of the word, then one load per further byte
while the node has children and the word has bytes (the last, failing lookup counted; a leaf or the
word's end stops without one).  With pair steps: one load per two bytes; a pair that misses needs the
one-byte lookup of the node between (its terminal flag), then the walk ends; one byte left: one load.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'tests'), os.path.join(ROOT, 'dp-tokenization_amd')]
from bloom_fixture import big_vocab
from dptok import synth
t2i = big_vocab()
toks = [t.encode('utf-8') for t in t2i]
term = set(toks)
pref = set()
for t in toks:
    for k in range(1, len(t) + 1): pref.add(t[:k])
haschild = set(t[:k] for t in toks for k in range(0, len(t)))   # prefixes with a longer token prefix
text, offs, cut = synth.bloom_like_parallel(int(sys.argv[1]) if len(sys.argv) > 1 else 20000, t2i, procs=8, length=256)
text = bytes(text); G = 64
single = pair = walks = 0
byts = 0
for s in range(len(offs) - 1):
    a, b = int(offs[s]), int(offs[s + 1])
    # words: cut[k]=1 where a word starts
    ws = [k for k in range(a, b) if cut[k] & 1] + [b]
    if not ws or ws[0] != a: ws = [a] + ws
    for wi in range(len(ws) - 1):
        w = text[ws[wi]:ws[wi + 1]]
        # atom starts: UTF-8 lead bytes
        starts = [k for k in range(len(w)) if (w[k] & 0xC0) != 0x80]
        for j in starts:
            walks += 1
            # single: bytes consumed via root table 2 (if >= 2 bytes left) then 1/step
            p = j; L = len(w)
            # matched prefix length in bytes: longest m such that w[j:j+m] in pref (stop at word end)
            m = 0
            while j + m < L and w[j:j + m + 1] in pref: m += 1
            # single-step loads
            if L - j >= 2:
                # root table covers 2 bytes: if m < 2 the walk ends there (root table says which exist)
                ls = 1
                if m >= 2:
                    cons = 2
                    # further steps: each consumes one byte; stops at leaf (no child) or word end or miss
                    while True:
                        node = w[j:j + cons]
                        if node not in haschild or j + cons >= L: break      # leaf or word end: no load
                        ls += 1
                        if w[j:j + cons + 1] in pref: cons += 1
                        else: break                                   # miss
            else:
                ls = 1
            single += ls
            # pair scheme
            if L - j >= 2:
                lp = 1
                if m >= 2:
                    cons = 2
                    while True:
                        node = w[j:j + cons]
                        if node not in haschild or j + cons >= L: break
                        if j + cons + 2 <= L:
                            lp += 1
                            if w[j:j + cons + 2] in pref: cons += 2; continue
                            # pair miss: the single step for the child (term flag), then end
                            lp += 1
                            break
                        else:
                            lp += 1
                            if w[j:j + cons + 1] in pref: cons += 1
                            break
            else:
                lp = 1
            pair += lp
print(f"walks {walks}: single-step loads {single/walks:.3f} per walk, pair-step loads {pair/walks:.3f}")
