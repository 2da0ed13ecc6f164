"""Per-call trace driver (GPU box): N raw-mode dp_tokenize(str) calls of one 256-byte string, for
`rocprofv3 --kernel-trace --memory-copy-trace` (tools/percall.py has the timings by layer).
Usage: python tools/percall_trace.py [N]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dp-tokenization_amd"), os.path.join(ROOT, "tests")]


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    from dptok import synth
    from fake_llama import FakeLlamaTokenizer
    from packages.tokenizer_utils import dp_tokenize_llama
    t2i = synth.llama_shaped_vocab()
    s = synth.unpack(*synth.random_ascii_corpus(1, 256, seed=1))[0]
    dp_tokenize, _ = dp_tokenize_llama(FakeLlamaTokenizer(t2i), "raw")
    for _ in range(n):
        dp_tokenize(s)
    print("calls", n)


if __name__ == "__main__":
    main()
