"""Diagnostic (GPU box): consecutive encode calls on one stream against two contexts on two streams (step k on
context / stream k % 2), so that a call's tail and finish pass overlap the next call's first pass.

    python tools/overlap_steps.py [n_strings ...]        (cfg2-shaped strings; default 125000 1000000)

Prints ms per call for both schedules and checks that every call's outputs equal the one-stream run's.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dp-tokenization_amd")]
import numpy as np  # noqa: E402

from dptok import Encoder, Vocab, synth  # noqa: E402


def main():
    sizes = [int(x) for x in sys.argv[1:]] or [125000, 1000000]
    import torch
    dev = torch.device("cuda", 0)
    vocab = Vocab(synth.llama_shaped_vocab(), 0)
    encs = [Encoder(vocab), Encoder(vocab)]
    streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
    for n in sizes:
        text, offs = synth.random_ascii_corpus(n, 256, seed=1)
        nb = int(offs[-1])
        dt = torch.from_numpy(text).to(dev)
        do = torch.from_numpy(offs.view(np.int64)).to(dev)
        outs = [(torch.empty(nb, dtype=torch.int32, device=dev), torch.empty(n + 1, dtype=torch.int64, device=dev),
                 torch.empty(n, dtype=torch.int32, device=dev)) for _ in range(2)]

        def call(i, s):
            ids, io, st = outs[i]
            encs[i].encode_device(dt.data_ptr(), nb, do.data_ptr(), n, ids.data_ptr(), nb, io.data_ptr(), st.data_ptr(),
                                  stream=streams[s].cuda_stream)

        K = 40 if n <= 250000 else 12
        res = {}
        for sched in ("one", "two", "one", "two"):
            for i in range(2):   # warm-up
                call(i, 0)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(streams[0])
            streams[1].wait_event(e0)
            for k in range(K):
                if sched == "one":
                    call(k % 2, 0)
                else:
                    call(k % 2, k % 2)
            done1 = torch.cuda.Event()
            done1.record(streams[1])
            streams[0].wait_event(done1)
            e1.record(streams[0])
            e1.synchronize()
            res.setdefault(sched, []).append(e0.elapsed_time(e1) / K)
        a, b = outs
        same = torch.equal(a[1], b[1]) and torch.equal(a[2], b[2]) and torch.equal(a[0][: int(a[1][-1])], b[0][: int(b[1][-1])])
        print(n, {k: [round(x, 4) for x in v] for k, v in res.items()},
              "GB/s one %.2f two %.2f" % (nb / min(res["one"]) / 1e6, nb / min(res["two"]) / 1e6), "outputs equal", same,
              flush=True)


if __name__ == "__main__":
    main()
