"""Probe (GPU box): can a copy of the CSR pass's size run UNDER the first tokenize pass?  Times, on cfg2
1M x 256 B: the first pass alone (dpt_encode_padded: no CSR pass), an LDS-free copy kernel alone
(torch int16 -> int32 over the staged-id volume, 2 B read + 4 B written per id, like the finish pass),
and both launched together on two streams.  If the pair takes about as long as the first pass alone,
a finish pass without LDS could hide behind the next call's first pass (DESIGN.md §9, next levers).
Usage: python tools/overlap_probe.py [reps]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dp-tokenization_amd")]


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    import numpy as np
    import torch
    from dptok import Encoder, Vocab, synth
    dev = torch.device("cuda", 0)
    text, offs = synth.random_ascii_corpus(1_000_000, 256, seed=1)
    enc = Encoder(Vocab(synth.llama_shaped_vocab(), 0))
    n_bytes, M = int(offs[-1]), len(offs) - 1
    d_text = torch.from_numpy(text).to(dev)
    d_off = torch.from_numpy(offs.view(np.int64)).to(dev)
    d_ids = torch.empty(n_bytes, dtype=torch.int32, device=dev)
    d_cnt = torch.empty(M, dtype=torch.int64, device=dev)
    d_st = torch.empty(M, dtype=torch.int32, device=dev)
    enc.reserve(n_bytes, M)
    n_ids = 209_000_000
    src = torch.ones(n_ids, dtype=torch.int16, device=dev)
    dst = torch.empty(n_ids, dtype=torch.int32, device=dev)
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)

    def tok(s):
        enc.encode_device_padded(d_text.data_ptr(), n_bytes, d_off.data_ptr(), M, d_ids.data_ptr(), n_bytes,
                                 d_cnt.data_ptr(), d_st.data_ptr(), stream=s.cuda_stream)

    def cp(s):
        with torch.cuda.stream(s):
            dst.copy_(src)

    def timed(f):
        for _ in range(2):
            f()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            f()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / reps * 1e3

    out = {"first_pass_ms": timed(lambda: tok(s1)), "copy_ms": timed(lambda: cp(s2))}
    out["serial_ms"] = timed(lambda: (tok(s1), cp(s1)))
    out["together_ms"] = timed(lambda: (tok(s1), cp(s2)))
    out["copy_first_ms"] = timed(lambda: (cp(s2), tok(s1)))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
