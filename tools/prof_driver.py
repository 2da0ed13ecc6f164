"""Minimal driver for rocprofv3 passes: R encodes of N cfg2 strings through the device path."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dp-tokenization_amd")]
import numpy as np
from dptok import synth
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
gen = sys.argv[3] if len(sys.argv) > 3 else "ascii"
# generated corpora are cached in /tmp (one GPU call runs this driver many times)
cache = "/tmp/dpt_corpus_%s_%d.npz" % (gen, n)
cut = None
if gen == "bloom":
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from bloom_fixture import big_vocab
    t2i = big_vocab()
else:
    t2i = synth.llama_shaped_vocab()
presplit = gen.endswith("p")   # ascii / s2orc in llama mode (bench --workload cfg2p / cfg4p): dptok.synth.llama_words
if presplit:
    gen = gen[:-1]
    cache = "/tmp/dpt_corpus_%s_%d.npz" % (gen, n)
if gen != "ascii" and os.path.exists(cache):
    z = np.load(cache)
    text, offs = z["text"], z["offs"]
    cut = z["cut"] if "cut" in z else None
elif gen == "ascii":
    text, offs = synth.random_ascii_corpus(n, 256, seed=1)
elif gen == "bloom":
    procs = 16 if (len(sys.argv) > 4 and sys.argv[4] == "gen-only") else 1
    text, offs, cut = synth.bloom_like_parallel(n, t2i, procs=procs, length=256)
    np.savez(cache, text=text, offs=offs, cut=cut)
else:
    # (forks: only in the gen-only run, which no profiler wraps)
    procs = 16 if (len(sys.argv) > 4 and sys.argv[4] == "gen-only") else 1
    text, offs = synth.generate_parallel("s2orc" if gen == "s2orc" else "arabic", n, procs=procs,
                                         **({"seed": 4} if gen == "s2orc" else {"length": 256, "seed": 5}))
    np.savez(cache, text=text, offs=offs)
if len(sys.argv) > 4 and sys.argv[4] == "gen-only":   # run without a profiler first: the forks happen here
    sys.exit(0)
if presplit:
    text, offs, cut = synth.llama_words(text, offs)
import torch  # noqa: E402
from dptok import Encoder, Vocab  # noqa: E402
enc = Encoder(Vocab(t2i, 0))
dev = torch.device("cuda", 0)
dt = torch.from_numpy(text).to(dev); do = torch.from_numpy(offs.view(np.int64)).to(dev)
nb = len(text)
ids = torch.empty(nb, dtype=torch.int32, device=dev); io = torch.empty(n + 1, dtype=torch.int64, device=dev)
st = torch.empty(n, dtype=torch.int32, device=dev)
s = torch.cuda.current_stream().cuda_stream
dc = torch.from_numpy(cut).to(dev) if cut is not None else None
for _ in range(reps):
    enc.encode_device(dt.data_ptr(), nb, do.data_ptr(), n, ids.data_ptr(), nb, io.data_ptr(), st.data_ptr(), stream=s,
                      cut_ptr=dc.data_ptr() if dc is not None else 0,
                      mode="presplit" if presplit else ("atoms" if dc is not None else "raw"))
torch.cuda.synchronize()
print("tokens", int(io[-1].item()), "bytes", nb)
