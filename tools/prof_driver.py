"""Minimal driver for rocprofv3 passes: R encodes of N cfg2 strings through the device path."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dp-tokenization_amd")]
import numpy as np
import torch
from dptok import Encoder, Vocab, synth
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
gen = sys.argv[3] if len(sys.argv) > 3 else "ascii"
enc = Encoder(Vocab(synth.llama_shaped_vocab(), 0))
if gen == "ascii":
    text, offs = synth.random_ascii_corpus(n, 256, seed=1)
elif gen == "s2orc":
    text, offs = synth.s2orc_like_corpus(n, seed=4)
else:
    text, offs = synth.arabic_corpus(n, 256, seed=5)
dev = torch.device("cuda", 0)
dt = torch.from_numpy(text).to(dev); do = torch.from_numpy(offs.view(np.int64)).to(dev)
nb = len(text)
ids = torch.empty(nb, dtype=torch.int32, device=dev); io = torch.empty(n + 1, dtype=torch.int64, device=dev)
st = torch.empty(n, dtype=torch.int32, device=dev)
s = torch.cuda.current_stream().cuda_stream
for _ in range(reps):
    enc.encode_device(dt.data_ptr(), nb, do.data_ptr(), n, ids.data_ptr(), nb, io.data_ptr(), st.data_ptr(), stream=s)
torch.cuda.synchronize()
print("tokens", int(io[-1].item()), "bytes", nb)
