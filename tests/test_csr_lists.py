"""The host path's CSR -> Python lists step (dptok/engine.py csr_lists, C extension _pylists) gives the
same (List[int], status) per string as the plain-Python conversion (the drop-in's return shape,
reference tokenizer_utils.py:66-80).  CPU only: no GPU call."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dp-tokenization_amd")]

from dptok import engine  # noqa: E402
from dptok import _lib  # noqa: E402


def _python(ids, id_off, st, none=None, keep_failed=True):
    saved = engine._pylists
    engine._pylists = None
    try:
        return engine.csr_lists(ids, id_off, st, none=none, keep_failed=keep_failed)
    finally:
        engine._pylists = saved


def test_extension_built():
    assert engine._pylists is not None, "build() compiles dptok/_pylists (csrc/Makefile)"


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_csr_lists_matches_python(seed):
    rng = np.random.default_rng(seed)
    n = int(rng.integers(0, 600))
    counts = rng.integers(0, 40, size=n)
    st = rng.choice([0, 0, 0, 1, 2, 3], size=n).astype(np.int32)
    counts[st != 0] = 0                       # failed strings carry no ids (the kernels' rule)
    id_off = np.zeros(n + 1, dtype=np.uint64)
    id_off[1:] = np.cumsum(counts)
    hi = [32000, 250680, 1 << 23][seed]       # past the C cache's range too
    ids = rng.integers(0, hi, size=int(id_off[-1])).astype(np.int32)
    none = rng.random(n) < 0.1
    for kf in (True, False):
        for nn in (None, none):
            got = engine.csr_lists(ids, id_off, st, none=nn, keep_failed=kf)
            assert got == _python(ids, id_off, st, none=nn, keep_failed=kf)
    got = engine.csr_lists(ids, id_off, st, none=none, keep_failed=False)
    for i in range(n):
        if none[i]:
            assert got[i] == ([], _lib.STATUS_OK)
        elif st[i] != 0:
            assert got[i] == ([], int(st[i]))
        else:
            assert got[i][0] == ids[int(id_off[i]):int(id_off[i + 1])].tolist()


def test_csr_lists_checks_offsets():
    ids = np.arange(4, dtype=np.int32)
    with pytest.raises(ValueError):
        engine.csr_lists(ids, np.array([0, 9], dtype=np.uint64), np.zeros(1, np.int32))
    assert engine.csr_lists(np.zeros(0, np.int32), np.zeros(1, np.uint64), np.zeros(0, np.int32)) == []
