import gzip
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "dp-tokenization_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs via gpurun)")
    config.addinivalue_line("markers", "slow: longer CPU tests")


def load_golden(name):
    path = os.path.join(GOLDEN, name)
    if name.endswith(".gz"):
        with gzip.open(path, "rt", encoding="utf-8") as f:
            return json.load(f)
    with open(path, encoding="utf-8") as f:
        return json.load(f)


CORPUS_FIXTURES = ["edge_llama32k.json.gz", "edge_toy1k.json.gz", "cfg1_toy1k.json.gz",
                   "cfg2_llama32k.json.gz", "cfg4_s2orc.json.gz", "cfg5_arabic.json.gz", "oov_llama32k.json.gz"]


@pytest.fixture(scope="session")
def vocabs():
    from dptok import synth
    return {"llama32k": synth.llama_shaped_vocab(), "toy1k": synth.toy_vocab()}


def vocab_sha(t2i):
    """Same checksum recipe as tests/golden/make_golden.py."""
    import hashlib
    return hashlib.sha256(json.dumps(list(t2i.items()), ensure_ascii=False).encode()).hexdigest()
