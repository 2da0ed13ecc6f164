"""Diagnostic: per-phase cycle shares of the tokenize kernel (libdpt_stamps.so build)."""
import ctypes, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["DPT_LIB"] = os.path.join(ROOT, "dp-tokenization_amd/csrc/build/libdpt_stamps.so")
sys.path[:0] = [ROOT, os.path.join(ROOT, "dp-tokenization_amd")]
import numpy as np
from dptok import Encoder, Vocab, synth, _lib
n = int(sys.argv[1]) if len(sys.argv) > 1 else 200000
L = int(sys.argv[2]) if len(sys.argv) > 2 else 256
gen = sys.argv[3] if len(sys.argv) > 3 else "ascii"
mode, cut = "raw", None
if gen == "bloom":   # the 250,680-token byte-level vocabulary, ATOMS mode (tools/prof_driver.py's setup)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from bloom_fixture import big_vocab
    enc = Encoder(Vocab(big_vocab(), 0))
    mode = "atoms"
else:
    enc = Encoder(Vocab(synth.llama_shaped_vocab(), 0))
cache = "/tmp/dpt_corpus_%s_%d.npz" % (gen, n)   # tools/prof_driver.py's gen-only cache
if gen != "ascii" and os.path.exists(cache):
    z = np.load(cache)
    text, offs = z["text"], z["offs"]
    cut = z["cut"] if "cut" in z else None
elif gen == "ascii":
    text, offs = synth.random_ascii_corpus(n, L, seed=1)
elif gen == "s2orc":
    text, offs = synth.s2orc_like_corpus(n, seed=4)
else:
    text, offs = synth.arabic_corpus(n, L, seed=5)
enc.encode_csr(text, offs, mode=mode, cut_mask=cut)
buf = (ctypes.c_ulonglong * 10)()
lib = _lib.lib()
lib.dpt_debug_stamps(buf, 1)
reps = int(os.environ.get("STAMP_REPS", "1"))   # (one-string calls: average over many)
t0 = time.time()
for _ in range(reps):
    enc.encode_csr(text, offs, mode=mode, cut_mask=cut)
dt = (time.time() - t0) / reps
lib.dpt_debug_stamps(buf, 0)
names = ["prep", "A_match", "B_forward", "C0/C1_select", "finish", "C2_bulk", "C2_hash", "C2_pend+walk",
         "(unused)", "tail"]
tot = sum(buf[k] for k in range(10))
print(f"{gen} n={n} wall={dt*1e3:.1f} ms (host path incl. copies)")
for k in (0, 1, 2, 3, 5, 6, 7, 4, 8, 9):
    print(f"  {names[k]:12s} {buf[k]/tot*100:6.2f}%  {buf[k]/n/reps:10.0f} cycles/string(wave)")
