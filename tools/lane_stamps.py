"""Diagnostic: forward vs backtrace cycles of the lane kernel (libdpt_stamps.so build)."""
import ctypes, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["DPT_LIB"] = os.path.join(ROOT, "dp-tokenization_amd/csrc/build/libdpt_stamps.so")
sys.path[:0] = [ROOT, os.path.join(ROOT, "dp-tokenization_amd")]
from dptok import Encoder, Vocab, synth, _lib
n = int(sys.argv[1]) if len(sys.argv) > 1 else 262144
enc = Encoder(Vocab(synth.llama_shaped_vocab(), 0))
text, offs = synth.random_ascii_corpus(n, 256, seed=1)
enc.encode_csr(text, offs)
buf = (ctypes.c_ulonglong * 4)()
lib = _lib.lib()
lib.dpt_debug_lane_stamps(buf, 1)
enc.encode_csr(text, offs)
lib.dpt_debug_lane_stamps(buf, 0)
w = buf[2]
print(f"waves={w} forward {buf[0]/w:.0f} cycles/wave  backtrace {buf[1]/w:.0f} cycles/wave  (64 strings per wave)")
