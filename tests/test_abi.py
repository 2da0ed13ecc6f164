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
    assert L.dpt_abi_version() == 1


def test_errors_without_device_or_args():
    import torch
    from dptok import _lib
    L = _lib.lib()
    h = ctypes.c_void_p()
    rc = L.dpt_ctx_create(0, None)
    assert rc == -1
    rc = L.dpt_vocab_create(None, None, None, 0, 0, ctypes.byref(h))
    assert rc == -1 and L.dpt_last_error()
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
