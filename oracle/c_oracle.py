"""ORACLE — test infrastructure only.  ctypes + numpy front end for oracle/hgin_oracle.c.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use it (as the checker).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "liboracle.so")
_lib = None


def build() -> str:
    src = os.path.join(HERE, "hgin_oracle.c")
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(src):
        subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB


def lib():
    global _lib
    if _lib is None:
        _lib = ctypes.CDLL(build())
        P = ctypes.c_void_p
        I64 = ctypes.c_int64
        _lib.oracle_csr_build.argtypes = [P, I64, ctypes.c_int, I64, I64, P, P, P]
        _lib.oracle_csr_build.restype = ctypes.c_int
        _lib.oracle_aggregate_f32.argtypes = [P, P, I64, P, I64, I64, P, I64, I64, ctypes.c_float, ctypes.c_int,
                                              P, I64]
        _lib.oracle_philox4x32_10.argtypes = [P, P, P]
        _lib.oracle_neg_sample.argtypes = [ctypes.c_uint64, ctypes.c_uint64, I64, I64, P]
        _lib.oracle_dot_decode_fwd_f32.argtypes = [P, P, I64, P, I64, P, I64, I64, P]
        _lib.oracle_dot_decode_bwd_f32.argtypes = [P, P, P, I64, P, P, I64, I64, P, I64]
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def csr_build(edge_index: np.ndarray, key_row: int, n_rows: int, n_cols: int):
    ei = np.ascontiguousarray(edge_index, dtype=np.int64)
    E = ei.shape[1]
    rowptr = np.zeros(n_rows + 1, np.int32)
    col = np.zeros(max(E, 1), np.int32)
    perm = np.zeros(max(E, 1), np.int32)
    st = lib().oracle_csr_build(_p(ei), E, key_row, n_rows, n_cols, _p(rowptr), _p(col), _p(perm))
    return rowptr, col[:E], perm[:E], st


def aggregate(rowptr, col, x_src: np.ndarray, x_dst, eps: float, mode: int) -> np.ndarray:
    x_src = np.ascontiguousarray(x_src, np.float32)
    n_rows = rowptr.shape[0] - 1
    f_src = x_src.shape[1]
    f_dst = 0 if x_dst is None else x_dst.shape[1]
    if x_dst is not None:
        x_dst = np.ascontiguousarray(x_dst, np.float32)
    width = f_src + (f_dst if mode == 2 else 0)
    out = np.zeros((n_rows, max(width, 1)), np.float32)
    col = np.ascontiguousarray(col, np.int32) if col.size else np.zeros(1, np.int32)
    lib().oracle_aggregate_f32(_p(np.ascontiguousarray(rowptr, np.int32)), _p(col), n_rows, _p(x_src),
                               max(f_src, 1), f_src, _p(x_dst), max(f_dst, 1), f_dst, float(eps), mode, _p(out),
                               out.shape[1])
    return out[:, :width]


def philox4x32_10(ctr, key):
    c = np.asarray(ctr, np.uint32)
    k = np.asarray(key, np.uint32)
    o = np.zeros(4, np.uint32)
    lib().oracle_philox4x32_10(_p(c), _p(k), _p(o))
    return o


def neg_sample(seed: int, offset: int, n: int, n_dst: int) -> np.ndarray:
    out = np.zeros(max(n, 1), np.int32)
    lib().oracle_neg_sample(seed, offset, n, n_dst, _p(out))
    return out[:n]


def dot_decode_fwd(src, dst, zs, zd) -> np.ndarray:
    src = np.ascontiguousarray(src, np.int32)
    dst = np.ascontiguousarray(dst, np.int32)
    zs = np.ascontiguousarray(zs, np.float32)
    zd = np.ascontiguousarray(zd, np.float32)
    out = np.zeros(max(len(src), 1), np.float32)
    lib().oracle_dot_decode_fwd_f32(_p(src), _p(dst), len(src), _p(zs), zs.shape[1], _p(zd), zd.shape[1],
                                    zs.shape[1], _p(out))
    return out[:len(src)]


def dot_decode_bwd(rowptr, col, perm, g, z_other) -> np.ndarray:
    n_rows = rowptr.shape[0] - 1
    zo = np.ascontiguousarray(z_other, np.float32)
    F = zo.shape[1]
    out = np.zeros((n_rows, max(F, 1)), np.float32)
    col = np.ascontiguousarray(col, np.int32) if len(col) else np.zeros(1, np.int32)
    perm = np.ascontiguousarray(perm, np.int32) if len(perm) else np.zeros(1, np.int32)
    lib().oracle_dot_decode_bwd_f32(_p(np.ascontiguousarray(rowptr, np.int32)), _p(col), _p(perm), n_rows,
                                    _p(np.ascontiguousarray(g, np.float32)), _p(zo), F, F, _p(out), out.shape[1])
    return out[:, :F]
