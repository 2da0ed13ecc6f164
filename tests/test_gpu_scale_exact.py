"""Bit-exactness at scale in the driver's GPU suite (the full-size exact checks of cfg4, cfg5
and BLOOM ran only on the builder's leases): the bench workloads' own corpora -- the same generators,
seeds and string indices as `bench.py --workload cfg4|cfg5|bloom` -- at the largest prefixes a
single-process generator makes in seconds, through the host path, every string's ids, offsets and
status against the C oracle (oracle/dp_oracle.c, OpenMP)."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

THREADS = max(1, min(16, os.cpu_count() or 1))


def _check(enc, ov, text, offs, mode, omode, cut=None):
    got = enc.encode_csr(text, offs, mode=mode, cut_mask=cut)
    ref = ov.encode_csr(text, offs, mode=omode, cut_mask=cut, nthreads=THREADS)
    for g, r, what in zip(got[:3], ref[:3], ("ids", "offsets", "status")):
        if not np.array_equal(g, r):
            bad = np.nonzero(np.asarray(g[: len(r)]) != np.asarray(r[: len(g)]))[0][:5]
            raise AssertionError((what, bad))
    return len(offs) - 1, int(offs[-1])


def test_cfg4_prefix_exact():
    """cfg4: the first 100,000 S2ORC-shaped abstracts of the bench corpus (~120 MB, half the bench run)."""
    from dptok import Encoder, Vocab, synth
    from oracle import oracle
    t2i = synth.llama_shaped_vocab()
    text, offs = synth.generate_parallel("s2orc", 100_000, start=0, procs=1, seed=4)
    n, nb = _check(Encoder(Vocab(t2i, 0)), oracle.OracleVocab(t2i), text, offs, "raw", oracle.RAW)
    assert n == 100_000 and nb > 100_000 * 600


def test_cfg5_prefix_exact():
    """cfg5: the first 250,000 Arabic-shaped strings of the bench corpus (~64 MB)."""
    from dptok import Encoder, Vocab, synth
    from oracle import oracle
    t2i = synth.llama_shaped_vocab()
    text, offs = synth.generate_parallel("arabic", 250_000, start=0, procs=1, length=256, seed=5)
    _check(Encoder(Vocab(t2i, 0)), oracle.OracleVocab(t2i), text, offs, "raw", oracle.RAW)


def test_bloom_prefix_exact():
    """BLOOM scale: the first 200,000 pre-tokenized byte-level strings of the bench corpus on the
    250,680-entry vocabulary (the 64-lane kernel, ATOMS mode)."""
    from bloom_fixture import big_vocab
    from dptok import Encoder, Vocab, synth
    from oracle import oracle
    t2i = big_vocab()
    text, offs, cut = synth.bloom_like_parallel(200_000, t2i, start=0, procs=1, length=256)
    _check(Encoder(Vocab(t2i, 0)), oracle.OracleVocab(t2i), text, offs, "atoms", oracle.ATOMS, cut)


def test_presplit_llama_mode_prefix_exact():
    """llama mode (pretokenize_option='llama', the factory's default, reference tokenizer_utils.py:52, :64-65) at
    bench scale: the first 262,144 cfg2 strings and 20,000 cfg4 abstracts of `bench.py --workload cfg2p|cfg4p`
    (BOS word + SentencePiece-shaped words, dptok.synth.llama_words), DPT_MODE_PRESPLIT, against the oracle's
    PRESPLIT mode -- every string."""
    from dptok import Encoder, Vocab, synth
    from oracle import oracle
    t2i = synth.llama_shaped_vocab()
    enc, ov = Encoder(Vocab(t2i, 0)), oracle.OracleVocab(t2i)
    text, offs = synth.random_ascii_corpus(262_144, 256, seed=1)
    t2, o2, cut = synth.llama_words(text, offs)
    n, nb = _check(enc, ov, t2, o2, "presplit", oracle.PRESPLIT, cut)
    assert n == 262_144 and nb > 262_144 * 262
    text, offs = synth.generate_parallel("s2orc", 20_000, start=0, procs=1, seed=4)
    t2, o2, cut = synth.llama_words(text, offs)
    _check(enc, ov, t2, o2, "presplit", oracle.PRESPLIT, cut)
