"""Where the per-call time of the drop-in goes (GPU box): one raw-mode dp_tokenize(str) call of a 256-byte
string, then the same work one layer down at a time -- Encoder.encode_strs, encode_csr (dpt_encode_host
through ctypes with numpy buffers), and dpt_encode on device buffers + a stream sync -- and the batch
form's stages (pack_strings, dpt_encode_host, csr_lists, the per-string status loop) for 4096 strings.
Usage: python tools/percall.py [reps]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dp-tokenization_amd"), os.path.join(ROOT, "tests")]


def per_call(f, reps):
    for _ in range(20):
        f()
    t0 = time.perf_counter()
    for _ in range(reps):
        f()
    return (time.perf_counter() - t0) / reps * 1e6


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
    import numpy as np
    import torch
    from dptok import engine, synth
    from fake_llama import FakeLlamaTokenizer
    from packages.tokenizer_utils import dp_tokenize_llama
    t2i = synth.llama_shaped_vocab()
    texts = synth.unpack(*synth.random_ascii_corpus(4096, 256, seed=1))
    s = texts[0]
    dp_tokenize, _ = dp_tokenize_llama(FakeLlamaTokenizer(t2i), "raw")
    enc = dp_tokenize.engine
    text1, offs1 = engine.pack_strings([s])
    out = {"dp_tokenize_us": per_call(lambda: dp_tokenize(s), reps),
           "encode_strs_us": per_call(lambda: enc.encode_strs([s]), reps),
           "encode_csr_us": per_call(lambda: enc.encode_csr(text1, offs1), reps),
           "pack_strings_us": per_call(lambda: engine.pack_strings([s]), reps)}
    dev = torch.device("cuda", 0)
    dt = torch.from_numpy(text1).to(dev)
    do = torch.from_numpy(offs1.view(np.int64)).to(dev)
    ids = torch.empty(len(text1), dtype=torch.int32, device=dev)
    io = torch.empty(2, dtype=torch.int64, device=dev)
    st = torch.empty(1, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream().cuda_stream

    def dev_call():
        enc.encode_device(dt.data_ptr(), len(text1) - 1, do.data_ptr(), 1, ids.data_ptr(), len(text1), io.data_ptr(),
                          st.data_ptr(), stream=stream)
        torch.cuda.synchronize()
    out["dpt_encode_device_sync_us"] = per_call(dev_call, reps)

    def sync_only():
        torch.cuda.synchronize()
    out["sync_only_us"] = per_call(sync_only, reps)
    # the batch form's stages
    k = 20
    t0 = time.perf_counter()
    for _ in range(k):
        text, offs = engine.pack_strings(texts)
    out["batch_pack_strings_ms"] = (time.perf_counter() - t0) / k * 1e3
    t0 = time.perf_counter()
    for _ in range(k):
        r = enc.encode_csr(text, offs)
    out["batch_encode_csr_ms"] = (time.perf_counter() - t0) / k * 1e3
    t0 = time.perf_counter()
    for _ in range(k):
        lists = engine.csr_lists(r[0], r[1], r[2])
    out["batch_csr_lists_ms"] = (time.perf_counter() - t0) / k * 1e3
    t0 = time.perf_counter()
    for _ in range(k):
        dp_tokenize.batch(texts)
    out["batch_total_ms"] = (time.perf_counter() - t0) / k * 1e3
    out["batch_bytes"] = int(offs[-1])
    print(json.dumps(out))


if __name__ == "__main__":
    main()
