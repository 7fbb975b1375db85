"""The C-ABI drop-in boundary: libhgin.so builds for gfx950, loads against torch's HIP runtime, exports
every entry point include/hgin.h declares, and rejects bad arguments before touching the device."""
import ctypes
import os
import re

import pytest

from conftest import ROOT
from hgin import _lib

HEADER = os.path.join(ROOT, "include", "hgin.h")


def declared_symbols():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|size_t|const char\*)\s+(hgin_\w+)\s*\(", text, re.M)))


def test_header_declares_the_bound_api():
    assert declared_symbols() == sorted(_lib.exported_symbols())


def test_library_exports_every_declared_symbol():
    lib = _lib.lib()
    for name in declared_symbols():
        assert hasattr(lib, name), name
    assert lib.hgin_abi_version() == _lib.ABI_VERSION


def test_single_hip_runtime_in_process():
    _lib.lib()
    maps = open("/proc/self/maps").read().splitlines()
    hip = sorted({l.split()[-1] for l in maps if "libamdhip64" in l})
    assert len(hip) == 1, hip


def test_argument_errors_do_not_touch_the_device():
    lib = _lib.lib()
    rc = lib.hgin_aggregate_f32(None, None, 10, None, 4, 4, None, 4, 4, None, 7, None, 4, None)
    assert rc == -1 and b"combine" in lib.hgin_last_error()
    rc = lib.hgin_aggregate_f32(None, None, 10, None, 4, 4, None, 4, 8, None, 1, None, 4, None)
    assert rc == -1  # ADD with f_dst != f_src (x_dst NULL also caught)
    rc = lib.hgin_csr_build(None, -1, 1, 5, 5, None, None, None, None, None, 0, None)
    assert rc == -1
    rc = lib.hgin_neg_sample(0, 0, 10, 0, None, None)
    assert rc == -1 and b"n_dst" in lib.hgin_last_error()
    rc = lib.hgin_gemm_nt_f32(None, 2, None, 2, None, 2, 4, 4, 4, None, None)
    assert rc == -1
    sz = ctypes.c_size_t(0)
    assert lib.hgin_csr_workspace_size(1000, 10, ctypes.byref(sz)) == 0 and sz.value >= 16000
    assert lib.hgin_csr_workspace_size(1000, 10, None) == -1


def test_workspace_too_small_is_reported():
    lib = _lib.lib()
    rc = lib.hgin_csr_build(ctypes.c_void_p(16), 100, 1, 5, 5, ctypes.c_void_p(16), ctypes.c_void_p(16),
                            None, ctypes.c_void_p(16), ctypes.c_void_p(16), 8, None)
    assert rc == -3 and b"workspace" in lib.hgin_last_error()


def test_build_is_gfx950_code_object():
    path = _lib.build()
    data = open(path, "rb").read()
    assert b"gfx950" in data
