"""Self-copy (round 4, an experiment: opt-in, compiled into csrc/Makefile's `sc` build only): the first
tokenize pass copies each finished string's ids into the CSR arrays itself once the first id of its
256-string batch is known (dpt_kernels.hip sc_prefix / sc_copy_run); the finish pass writes every
offset and copies only the batches it did not copy whole.  With the product library (no self-copy) the
cases still run as parity tests of the finish paths; test_self_copy_build runs this module again in a
child process on build/var_sc/libdpt.so (DPT_LIB) when that library was built.  Every case is checked bit-exact
against the C oracle AND against the same call with the self-copy switched off (DPT_SELF_COPY=0, the
fold / scan finish paths), and dpt_ctx_copy_stats shows how much the first pass did.  The cases are
built to reach the fallbacks: strings routed to the 2048-byte and unbounded passes at the start, in
the middle and at the end of the batch (no batch from a routed string on may be published in the
first pass), strings without ids (status 1 / 2), multi-window strings (queues that fill), and a
sequence of calls of alternating sizes on one context (the two parity regions of the batch arrays)."""
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng(vocabs):
    from dptok import Encoder, Vocab
    from oracle import oracle
    return {k: (Encoder(Vocab(v, 0)), oracle.OracleVocab(v)) for k, v in vocabs.items()}


def _run(enc, text, offs, sc: bool):
    old = os.environ.get("DPT_SELF_COPY")
    os.environ["DPT_SELF_COPY"] = "1" if sc else "0"
    try:
        out = enc.encode_csr(text, offs)
    finally:
        if old is None:
            os.environ.pop("DPT_SELF_COPY", None)
        else:
            os.environ["DPT_SELF_COPY"] = old
    return out, enc.copy_stats()


def _same(a, b, what):
    assert np.array_equal(a[2], b[2]), (what, "status", np.nonzero(a[2] != b[2])[0][:10])
    assert np.array_equal(a[1], b[1]), (what, "offsets", np.nonzero(a[1] != b[1])[0][:10])
    assert np.array_equal(a[0], b[0]), (what, "ids")


def _available():
    from dptok import _lib
    return bool(_lib.lib().dpt_self_copy_available())


def _check(e, text, offs, min_copied_frac=None):
    enc, orc = e
    on, st_on = _run(enc, text, offs, True)
    off, st_off = _run(enc, text, offs, False)
    ref = orc.encode_csr(text, offs)
    _same(on, ref, "self-copy vs oracle")
    _same(off, ref, "finish-only vs oracle")
    assert np.array_equal(on[3], ref[3])
    n = len(offs) - 1
    nb = (n + 255) // 256
    assert st_off == (0, 0, 0)
    if not _available():
        assert st_on == (0, 0, 0)
    elif nb >= 8:
        assert st_on[2] == nb, st_on
        if min_copied_frac is not None:
            assert st_on[0] >= min_copied_frac * n, (st_on, n)
    return st_on


def test_cfg2_shape_all_copied(eng):
    from dptok import synth
    text, offs = synth.random_ascii_corpus(50000, 256, seed=101)
    st = _check(eng["llama32k"], text, offs, min_copied_frac=0.9)
    print("cfg2 50k: copied %d of 50000, batches with offsets %d of %d" % st)


def test_s2orc_and_arabic(eng):
    from dptok import synth
    for text, offs in (synth.s2orc_like_corpus(3000, seed=7), synth.arabic_corpus(30000, seed=8)):
        st = _check(eng["llama32k"], text, offs, min_copied_frac=0.5)
        print("copied %d, batches %d of %d" % st)


@pytest.mark.parametrize("where", ["first", "middle", "last", "many"])
def test_routed_strings_block_publication(eng, where):
    """A string with a word over 256 bytes goes to the 2048-byte pass (over 2048: the unbounded
    pass); the first pass may not publish its batch or any later one."""
    from dptok import pack_strings, synth
    rng = np.random.default_rng({"first": 1, "middle": 2, "last": 3, "many": 4}[where])
    text, offs = synth.random_ascii_corpus(6000, 200, seed=9)
    texts = [bytes(text[int(offs[i]):int(offs[i + 1])]).decode("ascii") for i in range(6000)]
    pos = {"first": [0], "middle": [3000], "last": [5999], "many": [17, 2500, 2511, 4100]}[where]
    for k, p in enumerate(pos):
        L = 300 if k % 2 == 0 else 2500
        texts[p] = "ab " + "".join(chr(c) for c in rng.integers(0x21, 0x7F, size=L)) + " cd"
    t, o = pack_strings(texts)
    st = _check(eng["llama32k"], t, o)
    first = min(pos) // 256
    # nothing from the first routed string's batch on was copied by the first pass (that batch never
    # completes there, so no later batch learns its first id)
    assert st[1] <= first and st[0] <= first * 256, (st, first)


def test_strings_without_ids(eng):
    """status 1 (no tokenization: the toy vocabulary lacks many characters) and status 2 (empty)
    strings finish with no ids: counted as copied at once, never queued."""
    from dptok import pack_strings
    rng = np.random.default_rng(12)
    pool = [chr(c) for c in range(0x21, 0x7F)] + ["é", "中", "\n", " "] * 3
    texts = []
    for i in range(5000):
        r = i % 7
        texts.append("" if r == 0 else "".join(rng.choice(pool, size=int(rng.integers(1, 120)))))
    t, o = pack_strings(texts)
    for name in ("toy1k", "llama32k"):
        _check(eng[name], t, o)


def test_calls_of_alternating_sizes(eng):
    """One context, calls alternating between self-copy, fold, scan and one-batch sizes: each call
    must leave the next parity's region zeroed."""
    from dptok import synth
    enc, orc = eng["llama32k"]
    big = 256 * 2048 + 300   # > FIN_FOLD_MAX batches (the finish-only path would scan)
    text_all, offs_all = synth.random_ascii_corpus(big, 20, seed=77)
    for k, n in enumerate([5000, 2048, 300, big, 2047, 40000, 1, 2100, big, 600, 5000]):
        a = (k * 1231) % (big - n + 1)
        offs = (offs_all[a:a + n + 1] - offs_all[a]).astype(np.uint64)
        text = np.ascontiguousarray(text_all[int(offs_all[a]):int(offs_all[a + n])])
        got, st = _run(enc, text, offs, True)
        _same(got, orc.encode_csr(text, offs), ("call", k, n))
        nb = (n + 255) // 256
        assert (st[2] == nb) == (nb >= 8 and _available()), (k, n, st)


def test_self_copy_build():
    """This module on the self-copy build (csrc/Makefile `sc`), in one child process."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    lib = os.path.join(root, "dp-tokenization_amd", "csrc", "build", "var_sc", "libdpt.so")
    if _available() or os.environ.get("DPT_LIB"):
        pytest.skip("already running on a self-copy build")
    if not os.path.exists(lib):
        pytest.skip("build/var_sc/libdpt.so not built (make -C dp-tokenization_amd/csrc sc)")
    env = dict(os.environ, DPT_LIB=lib)
    r = subprocess.run([sys.executable, "-m", "pytest", "-x", "-q", "-m", "gpu", "-p", "no:cacheprovider",
                        os.path.abspath(__file__), "--timeout", "150", "--timeout-method", "thread"],
                       cwd=root, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
