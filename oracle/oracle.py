"""TEST INFRASTRUCTURE ONLY -- ctypes wrapper around the C oracle (dp_oracle.c).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline /
exact-match leg may import this module.  The product package
(``dp-tokenization_amd/``) never does: it fails loudly without its HIP library.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")

RAW, PRESPLIT, ATOMS = 0, 1, 2


def build(force: bool = False) -> str:
    src = os.path.join(HERE, "dp_oracle.c")
    if force or not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(src):
        subprocess.check_call(["make", "-s", "-C", HERE, "liboracle.so"])
    return LIB


_lib = None


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(LIB)
        L.orc_vocab_new.restype = ctypes.c_void_p
        L.orc_vocab_new.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32]
        L.orc_vocab_free.argtypes = [ctypes.c_void_p]
        L.orc_encode.restype = ctypes.c_int
        L.orc_encode.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                 ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64,
                                 ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        _lib = L
    return _lib


def _ptr(a: Optional[np.ndarray]):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def pack_vocab(t2i: Dict[str, int]) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    toks = list(t2i.keys())
    enc = [t.encode("utf-8", "surrogatepass") for t in toks]
    off = np.zeros(len(enc) + 1, dtype=np.uint64)
    off[1:] = np.cumsum([len(e) for e in enc], dtype=np.uint64)
    blob = np.frombuffer(b"".join(enc) or b"\0", dtype=np.uint8).copy()
    ids = np.array([t2i[t] for t in toks], dtype=np.int32)
    return blob, off, ids


class OracleVocab:
    def __init__(self, t2i: Dict[str, int]):
        self._blob, self._off, self._ids = pack_vocab(t2i)
        self.h = lib().orc_vocab_new(_ptr(self._blob), _ptr(self._off), _ptr(self._ids), len(self._ids))

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.orc_vocab_free(self.h)
            self.h = None

    def encode_csr(self, text: np.ndarray, offs: np.ndarray, mode: int = RAW,
                   cut_mask: Optional[np.ndarray] = None, nthreads: int = 0):
        """-> (ids int32[], id_off u64[n+1], status int32[n], capped_len int32[n])."""
        n = len(offs) - 1
        text = np.ascontiguousarray(text, dtype=np.uint8)
        offs = np.ascontiguousarray(offs, dtype=np.uint64)
        cap = int(offs[-1] - offs[0])
        ids = np.empty(max(cap, 1), dtype=np.int32)
        id_off = np.empty(n + 1, dtype=np.uint64)
        status = np.empty(max(n, 1), dtype=np.int32)
        capped = np.empty(max(n, 1), dtype=np.int32)
        if cut_mask is not None:
            cut_mask = np.ascontiguousarray(cut_mask, dtype=np.uint8)
        rc = lib().orc_encode(self.h, mode, _ptr(text), _ptr(offs), _ptr(cut_mask), n, _ptr(ids),
                              max(cap, 1), _ptr(id_off), _ptr(status), _ptr(capped), nthreads)
        if rc != 0:
            raise RuntimeError("orc_encode failed: %d" % rc)
        return ids[: int(id_off[-1])], id_off, status[:n], capped[:n]

    def encode_strs(self, texts: Sequence[str], nthreads: int = 0) -> List[Tuple[List[int], int]]:
        enc = [t.encode("utf-8", "surrogatepass") for t in texts]
        offs = np.zeros(len(enc) + 1, dtype=np.uint64)
        offs[1:] = np.cumsum([len(e) for e in enc], dtype=np.uint64)
        text = np.frombuffer(b"".join(enc) or b"\0", dtype=np.uint8)
        ids, id_off, st, _ = self.encode_csr(text, offs, nthreads=nthreads)
        return [(ids[int(id_off[i]):int(id_off[i + 1])].tolist(), int(st[i])) for i in range(len(enc))]
