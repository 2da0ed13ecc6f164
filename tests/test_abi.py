"""CPU checks of the C-ABI boundary: libdpt.so loads, exports every symbol that
include/dpt.h declares, and reports errors (no GPU needed)."""
import ctypes
import os
import re

import pytest

from conftest import PKG, ROOT


def _declared():
    src = open(os.path.join(ROOT, "include", "dpt.h")).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(dpt_\w+)\s*\(", src, re.M)))


def test_header_declares_expected_api():
    names = _declared()
    for must in ("dpt_vocab_create", "dpt_vocab_destroy", "dpt_encode", "dpt_encode_host", "dpt_token_histogram",
                 "dpt_last_error", "dpt_ctx_create"):
        assert must in names


def test_library_exports_every_declared_symbol():
    from dptok import _lib
    L = _lib.lib()
    for name in _declared():
        assert hasattr(L, name), name
    assert set(_declared()) == set(_lib.EXPORTED)
    assert L.dpt_abi_version() == 6
    for gone in ("dpt_ctx_pipeline", "dpt_ctx_join", "dpt_ctx_copy_stats", "dpt_self_copy_available"):   # ABI 4 dropped them
        assert not hasattr(L, gone), gone


def test_errors_without_device_or_args():
    import torch
    from dptok import _lib
    L = _lib.lib()
    h = ctypes.c_void_p()
    rc = L.dpt_ctx_create(0, None)
    assert rc == -1
    rc = L.dpt_vocab_create(None, None, None, 0, 0, ctypes.byref(h))
    assert rc == -1 and L.dpt_last_error()
    # dpt_encode_padded checks its arguments before any device work: null ctx / vocab, null counts
    off0 = (ctypes.c_uint64 * 1)(0)
    assert L.dpt_encode_padded(None, None, 0, None, 0, off0, None, 0, None, 0, None, None, None, None) == -1
    assert b"counts" in L.dpt_last_error()
    if not torch.cuda.is_available():
        off = (ctypes.c_uint64 * 2)(0, 1)
        blob = ctypes.create_string_buffer(b"a")
        rc = L.dpt_vocab_create(blob, off, None, 1, 0, ctypes.byref(h))
        assert rc == -5, L.dpt_last_error()


def test_product_path_has_no_cpu_fallback():
    """The package must not import the oracle anywhere."""
    for dp, _, fs in os.walk(PKG):
        for f in fs:
            if f.endswith(".py"):
                src = open(os.path.join(dp, f), encoding="utf-8").read()
                assert "oracle" not in src.replace("no CPU fallback", ""), os.path.join(dp, f)


def test_host_path_rejects_bad_offsets():
    """dpt_encode_host validates offsets before touching a device (a backwards offset
    would wrap the kernel's 32-bit string length and read past the text)."""
    from dptok import _lib
    L = _lib.lib()
    text = ctypes.create_string_buffer(b"abcdef")
    ids = (ctypes.c_int32 * 8)()
    id_off = (ctypes.c_uint64 * 4)()
    status = (ctypes.c_int32 * 3)()
    # 0 -> 4 -> 2 -> 6: sums to n_bytes = 6 but goes backwards
    off = (ctypes.c_uint64 * 4)(0, 4, 2, 6)
    rc = L.dpt_encode_host(None, None, 0, text, 6, off, None, 3, ids, 8, id_off, status, None)
    assert rc == -1 and b"monotone" in L.dpt_last_error()
    big = (ctypes.c_uint64 * 3)(0, 1 << 32, (1 << 32) + 6)
    rc = L.dpt_encode_host(None, None, 0, text, (1 << 32) + 6, big, None, 2, ids, (1 << 32) + 6, id_off, status, None)
    assert rc == -1 and b"4 GiB" in L.dpt_last_error()
    ok = (ctypes.c_uint64 * 4)(0, 2, 4, 6)
    rc = L.dpt_encode_host(None, None, 0, text, 6, ok, None, 3, ids, 8, id_off, status, None)
    assert rc == -1 and b"null ctx" in L.dpt_last_error()


def test_rccl_entry_points_check_arguments():
    """ABI 6 (SURVEY.md §8(b) dpt_hist_allreduce): argument errors before RCCL or a device is touched."""
    from dptok import _lib
    L = _lib.lib()
    comm = ctypes.c_void_p()
    idb = (ctypes.c_uint8 * _lib.DPT_RCCL_ID_BYTES)()
    assert L.dpt_rccl_get_unique_id(None) == -1
    assert L.dpt_hist_allreduce(None, 4, None, None) == -1 and b"null" in L.dpt_last_error()
    for world, rank, dev in ((0, 0, 0), (2, 2, 0), (2, -1, 0), (1, 0, -1)):
        assert L.dpt_rccl_comm_create(idb, world, rank, dev, ctypes.byref(comm)) == -1
    assert L.dpt_rccl_comm_create(None, 1, 0, 0, ctypes.byref(comm)) == -1
    assert L.dpt_rccl_comm_destroy(None) == 0
