"""Host logic of bench.py: the exact-match count (vectorised path and per-string fallback)."""
import os
import sys

import numpy as np

from conftest import ROOT

sys.path.insert(0, ROOT)
import bench  # noqa: E402  (no GPU work at import)


def _csr(rows):
    off = np.zeros(len(rows) + 1, dtype=np.uint64)
    off[1:] = np.cumsum([len(r) for r in rows])
    ids = np.concatenate([np.asarray(r, dtype=np.int32) for r in rows]) if rows else np.zeros(0, np.int32)
    return ids, off


def _loop(a, b, S):
    return sum(int(a[2][i] == b[2][i] and np.array_equal(a[0][int(a[1][i]):int(a[1][i + 1])], b[0][int(b[1][i]):int(b[1][i + 1])]))
               for i in range(S))


def test_exact_matches_vectorised_and_fallback():
    rng = np.random.default_rng(3)
    rows = [rng.integers(0, 32000, size=int(rng.integers(0, 9))).tolist() for _ in range(500)]
    ids, off = _csr(rows)
    st = np.zeros(500, dtype=np.int32)
    ref = (ids.copy(), off.copy(), st.copy())
    # identical
    assert bench.exact_matches(ids, off, st, *ref, 500) == 500
    # same counts, a few wrong ids and one wrong status: the vectorised path
    ids2 = ids.copy()
    hit = rng.choice(len(ids2), 7, replace=False)
    ids2[hit] += 1
    st2 = st.copy()
    st2[11] = 2
    got = (ids2, off, st2)
    assert bench.exact_matches(*got, *ref, 500) == _loop(got, ref, 500)
    # a count differs: the per-string fallback
    rows3 = [r[:] for r in rows]
    k = next(i for i, r in enumerate(rows3) if r)
    rows3[k] = rows3[k][:-1]
    ids3, off3 = _csr(rows3)
    got3 = (ids3, off3, st)
    assert bench.exact_matches(*got3, *ref, 500) == 499 == _loop(got3, ref, 500)
    # a prefix sample
    assert bench.exact_matches(*got, *ref, 100) == _loop(got, ref, 100)


def test_strong_shards_tile_the_corpus():
    """cfg3 (BASELINE configs[2]): rank r of W takes [r*N/W, (r+1)*N/W) of ONE corpus."""
    for n in (1, 7, 125_000, 1_000_000, 1_000_003):
        for w in (1, 2, 4, 8):
            r = [bench.rank_strings(n, k, w, "strong") for k in range(w)]
            assert r[0][0] == 0 and r[-1][1] == n
            assert all(r[k][1] == r[k + 1][0] for k in range(w - 1))
            assert sum(b - a for a, b in r) == n
    # weak: every rank owns its own n strings of the global index space, disjoint
    r = [bench.rank_strings(1000, k, 4, "weak") for k in range(4)]
    assert r == [(0, 1000), (1000, 2000), (2000, 3000), (3000, 4000)]


def test_batches_in_flight_rule():
    """--inflight: as given, else four batches in flight for the strong-scaling shards of 65,536.. strings and
    <= 64 MiB of text (125k / 250k x 256 B at 8 / 4 ranks), three for other shards of <= 524,288 strings (500k at 2
    ranks, cfg4's 200k S2ORC-shaped strings, cfg1) and one for the 1M single-GPU line."""
    b = lambda n, nb=None, **kw: bench.batches_in_flight(0, n, n_bytes=256 * n if nb is None else nb, **kw)  # noqa: E731
    assert b(125_000) == 4 and b(250_000) == 4
    assert b(500_000) == 3 and b(200_000, 245_000_000) == 3 and b(1000, 64_000) == 3
    assert b(1_000_000) == 1
    assert bench.batches_in_flight(1, 125_000) == 1
    assert bench.batches_in_flight(2, 1_000_000) == 2
    shard = [bench.rank_strings(1_000_000, 0, w, "strong") for w in (1, 2, 4, 8)]
    assert [b(hi - lo) for lo, hi in shard] == [1, 3, 4, 4]
    assert b(250_000, rows64=True) == 1   # BLOOM's 64-lane kernel


def test_algorithmic_bytes_follow_survey_8d():
    # cfg2: 1M x 256 B, tau = 0.816 ids/byte -> ~1.11 GB per launch with ids at 4 bytes
    n_str, n_bytes = 1_000_000, 256_000_000
    n_tok = int(0.816 * n_bytes)
    b = bench.algorithmic_bytes(n_bytes, n_str, n_tok)
    assert b == n_bytes + 4 * n_tok + 8 * (n_str + 1) * 2 + 4 * n_str
    assert 1.10e9 < b < 1.12e9
    assert bench.algorithmic_bytes(n_bytes, n_str, n_tok, 2) == b - 2 * n_tok


def test_cpu_share_reports_threads_used(monkeypatch):
    monkeypatch.setenv("OMP_NUM_THREADS", "3")
    used, vis = bench.cpu_share()
    assert used == min(3, vis) and vis >= 1
    monkeypatch.delenv("OMP_NUM_THREADS")
    used, vis = bench.cpu_share()
    assert used == vis


def test_words_of_atoms_round_trip():
    """bench.py's atoms-mode unpacking (the bloom workload's CPU-baseline input) inverts
    dptok.engine.pack_word_atoms, and the reference-port composition runs on it."""
    from dptok.engine import pack_word_atoms
    strings = [[["a", "b"], ["Ġ", "c", "é"]], [["x"]], [["Ġ", "Ġ"], ["😀", "z"], ["q"]]]
    text, offs, cut = pack_word_atoms(strings)
    assert bench.words_of_atoms(text, offs, cut) == strings
    from oracle import ref_port
    t2i = {"ab": 0, "Ġc": 1, "é": 2, "x": 3, "ĠĠ": 4, "😀z": 5, "q": 6, "a": 7, "b": 8, "Ġ": 9}
    assert ref_port.dp_tokenize_word_atoms(strings[0], t2i) == ([0, 1, 2], 0)
    assert ref_port.dp_tokenize_word_atoms(strings[2], t2i) == ([4, 5, 6], 0)


def test_gpus_flag_against_world_size():
    """--gpus N: run here at N = 1, launch the ranks (0) at N > 1 without torchrun, and refuse a
    torchrun job of another size (a silently smaller job would mis-measure the scaling run)."""
    import argparse
    import pytest
    ns = lambda g: argparse.Namespace(gpus=g)   # noqa: E731
    assert bench.resolve_world(ns(None), {}) == 1
    assert bench.resolve_world(ns(1), {}) == 1
    assert bench.resolve_world(ns(8), {}) == 0
    assert bench.resolve_world(ns(None), {"WORLD_SIZE": "4"}) == 4
    assert bench.resolve_world(ns(4), {"WORLD_SIZE": "4"}) == 4
    with pytest.raises(SystemExit) as e:
        bench.resolve_world(ns(8), {"WORLD_SIZE": "1"})
    assert e.value.code == 2
    with pytest.raises(SystemExit):
        bench.resolve_world(ns(2), {"WORLD_SIZE": "8"})


def test_bench_refuses_world_size_mismatch_in_a_child():
    """The refusal as a process: `WORLD_SIZE=1 python bench.py --gpus 8` exits 2 before any GPU work."""
    import subprocess
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8", "--no-cpu-baseline"],
                         env=env, capture_output=True, text=True, timeout=120)
    assert out.returncode == 2, out.stderr[-2000:]
    assert "WORLD_SIZE" in out.stderr and out.stdout.strip() == ""
