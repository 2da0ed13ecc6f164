"""Diagnostic (libdpt built with -DDPT_LANEDBG): per-lane chunk values of string 0."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["DPT_LIB"] = os.path.join(ROOT, "dp-tokenization_amd/csrc/build/var_dbg/libdpt.so")
sys.path[:0] = [ROOT, os.path.join(ROOT, "dp-tokenization_amd"), os.path.join(ROOT, "tests")]
from dptok import Encoder, Vocab, synth, _lib
from conftest import load_golden
g = load_golden("cfg2_llama32k.json.gz")
enc = Encoder(Vocab(synth.llama_shaped_vocab(), 0))
print(enc.encode_strs([g["cases"][int(sys.argv[1]) if len(sys.argv) > 1 else 6]["text"]])[0][0][100:110])
buf = (ctypes.c_uint * 260)()
_lib.lib().dpt_debug_lanes(buf)
names = "rs re pe T tb gin gre ls1 left fl fin_in n1 afin lsm flags in".split()
print("counts lanes/capless/capb", buf[258], buf[257], buf[256])
for d in range(16):
    print(d, {names[k]: buf[d * 16 + k] for k in range(16)})
