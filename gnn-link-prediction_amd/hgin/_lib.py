"""Build + ctypes binding of libhgin.so (the C ABI in include/hgin.h).

The library is compiled in-tree for gfx950 with hipcc (``build()``), so the shared object travels with the
repository snapshot to the GPU box.  Loading order matters: ``torch`` is imported first so that its bundled
HIP runtime (SONAME ``libamdhip64.so.7``) is the one libhgin.so binds to — one HIP runtime per process,
hence torch's device pointers and streams are valid in our kernels.

There is no fallback: if the library cannot be built or loaded, every op raises ``HginUnavailable``.
"""
from __future__ import annotations

import ctypes
import glob
import os
import shutil
import subprocess
import tempfile
import threading

import torch  # noqa: F401  (must be loaded before libhgin.so; see module docstring)

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG_DIR)                      # gnn-link-prediction_amd/
REPO = os.path.dirname(ROOT)
CSRC = os.path.join(ROOT, "csrc")
INCLUDE = os.path.join(REPO, "include")
BUILD_DIR = os.path.join(PKG_DIR, "_build")
LIB_PATH = os.path.join(BUILD_DIR, "libhgin.so")
ARCH = os.environ.get("HGIN_OFFLOAD_ARCH", "gfx950")
HIPCC_FLAGS = ["-O3", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off", f"--offload-arch={ARCH}"]

_lock = threading.Lock()
_lib = None


class HginUnavailable(RuntimeError):
    """libhgin.so (the HIP hot path) could not be built or loaded; there is no CPU fallback."""


class HginError(RuntimeError):
    """A libhgin.so entry point returned a non-zero status."""


def sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")))


def _deps():
    return sources() + sorted(glob.glob(os.path.join(CSRC, "*.h"))) + [os.path.join(INCLUDE, "hgin.h")]


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise HginUnavailable("hipcc not found (set HIPCC)")


def is_stale() -> bool:
    if not os.path.exists(LIB_PATH):
        return True
    t = os.path.getmtime(LIB_PATH)
    return any(os.path.getmtime(p) > t for p in _deps())


def _object(src: str) -> str:
    return os.path.join(BUILD_DIR, os.path.basename(src)[:-4] + ".o")


def _compile(src: str, verbose: bool) -> None:
    """One translation unit -> an object carrying its own gfx950 code object (no -fgpu-rdc: kernels never
    call across files), rebuilt only when it or a header changed."""
    obj = _object(src)
    headers = sorted(glob.glob(os.path.join(CSRC, "*.h"))) + [os.path.join(INCLUDE, "hgin.h")]
    if os.path.exists(obj) and all(os.path.getmtime(p) <= os.path.getmtime(obj) for p in [src] + headers):
        return
    tmp = obj + f".{os.getpid()}.tmp"
    cmd = [_hipcc()] + [f for f in HIPCC_FLAGS if f != "-shared"] + ["-I", INCLUDE, "-c", "-o", tmp, src]
    if verbose:
        print(" ".join(cmd))
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        if os.path.exists(tmp):
            os.unlink(tmp)
        raise HginUnavailable(f"hipcc failed on {os.path.basename(src)} ({res.returncode}):\n{res.stderr[-4000:]}")
    os.replace(tmp, obj)


def build(force: bool = False, verbose: bool = False) -> str:
    """Compile every HIP source for gfx950 (one object per file, in parallel) and link libhgin.so (atomic
    replace).  Returns the path."""
    if not force and not is_stale():
        return LIB_PATH
    from concurrent.futures import ThreadPoolExecutor
    os.makedirs(BUILD_DIR, exist_ok=True)
    srcs = sources()
    if force:
        for s in srcs:
            if os.path.exists(_object(s)):
                os.unlink(_object(s))
    jobs = max(1, min(len(srcs), int(os.environ.get("MAX_JOBS", "0") or 0) or (os.cpu_count() or 4), 16))
    with ThreadPoolExecutor(jobs) as ex:
        for f in [ex.submit(_compile, s, verbose) for s in srcs]:
            f.result()
    fd, tmp = tempfile.mkstemp(prefix=".libhgin.", suffix=".so", dir=BUILD_DIR)
    os.close(fd)
    cmd = [_hipcc(), "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", tmp] + [_object(s) for s in srcs]
    if verbose:
        print(" ".join(cmd))
    try:
        res = subprocess.run(cmd, capture_output=True, text=True)
        if res.returncode != 0:
            raise HginUnavailable(f"hipcc link failed ({res.returncode}):\n{res.stderr[-4000:]}")
        os.replace(tmp, LIB_PATH)
    finally:
        if os.path.exists(tmp):
            os.unlink(tmp)
    return LIB_PATH


_I64, _I32, _U64, _SZ = ctypes.c_int64, ctypes.c_int, ctypes.c_uint64, ctypes.c_size_t
_P = ctypes.c_void_p
_SIGS = {
    "hgin_abi_version": ([], _I32),
    "hgin_last_error": ([], ctypes.c_char_p),
    "hgin_csr_workspace_size": ([_I64, _I64, ctypes.POINTER(_SZ)], _I32),
    "hgin_csr_build": ([_P, _I64, _I32, _I64, _I64, _P, _P, _P, _P, _P, _SZ, _P], _I32),
    "hgin_aggregate_f32": ([_P, _P, _I64, _P, _I64, _I64, _P, _I64, _I64, _P, _I32, _P, _I64, _P], _I32),
    "hgin_combine_bwd_workspace_size": ([_I64, ctypes.POINTER(_SZ)], _I32),
    "hgin_combine_bwd_f32": ([_P, _I64, _P, _I64, _I64, _I64, _P, _P, _I64, _P, _P, _SZ, _P], _I32),
    "hgin_gin_mlp_fwd_f32": ([_P, _I64, _I64, _P, _I64, _P, _P, _P, _P, _P, _P, _P, _I64, _I64, _I64, _P, _P], _I32),
    "hgin_linear_fwd_f32": ([_P, _I64, _I64, _P, _I64, _P, _P, _P, _I64, _I64, _I64, _P, _P], _I32),
    "hgin_prelu_bwd_workspace_size": ([_I64, _I64, ctypes.POINTER(_SZ)], _I32),
    "hgin_prelu_bwd_f32": ([_P, _I64, _P, _I64, _I64, _P, _P, _P, _P, _P, _SZ, _P], _I32),
    "hgin_gemm_nt_f32": ([_P, _I64, _P, _I64, _P, _I64, _I64, _I64, _I64, _P, _P], _I32),
    "hgin_gemm_nt_combine_workspace_size": ([_I64, _I64, ctypes.POINTER(_SZ)], _I32),
    "hgin_gemm_nt_combine_f32": ([_P, _I64, _P, _I64, _P, _I64, _I64, _I64, _I64, _P, _I64, _P, _I64, _P, _I64, _I64,
                                  _P, _P, _P, _SZ, _P, _P], _I32),
    "hgin_gemm_nt_combine_bf16": ([_P, _I64, _P, _I64, _P, _I64, _I64, _I64, _I64, _P, _I64, _P, _I64, _P, _I64, _I64,
                                   _P, _P, _P, _SZ, _P, _P], _I32),
    "hgin_gemm_tn_workspace_size": ([_I64, _I64, _I64, ctypes.POINTER(_SZ)], _I32),
    "hgin_gemm_tn_f32": ([_P, _I64, _P, _I64, _I64, _P, _I64, _I64, _I64, _I64, _P, _I64, _P, _SZ, _P], _I32),
    "hgin_aggregate_bf16": ([_P, _P, _I64, _P, _I64, _I64, _P, _I64, _I64, _P, _I32, _P, _I64, _P], _I32),
    "hgin_gin_mlp_fwd_bf16": ([_P, _I64, _I64, _P, _I64, _P, _P, _P, _P, _P, _P, _P, _I64, _I64, _I64, _P, _P], _I32),
    "hgin_linear_fwd_bf16": ([_P, _I64, _I64, _P, _I64, _P, _P, _P, _I64, _I64, _I64, _P, _P], _I32),
    "hgin_gemm_nt_bf16": ([_P, _I64, _P, _I64, _P, _I64, _I64, _I64, _I64, _P, _P], _I32),
    "hgin_gemm_tn_bf16": ([_P, _I64, _P, _I64, _I64, _P, _I64, _I64, _I64, _I64, _P, _I64, _P, _SZ, _P], _I32),
    "hgin_prelu_bwd_bf16": ([_P, _I64, _P, _I64, _I64, _P, _P, _P, _P, _P, _SZ, _P], _I32),
    "hgin_gin_mlp_bwd_w_workspace_size": ([_I64, _I64, _I64, _I32, _I32, ctypes.POINTER(_SZ)], _I32),
    "hgin_gin_mlp_bwd_w_f32": ([_P, _I64, _P, _I64, _P, _P, _I64, _I64, _P, _I64, _I64, _I64, _I64, _P, _I64, _P, _P,
                                _P, _I64, _P, _SZ, _P], _I32),
    "hgin_gin_mlp_bwd_w_bf16": ([_P, _I64, _P, _I64, _P, _P, _I64, _I64, _P, _I64, _I64, _I64, _I64, _P, _I64, _P, _P,
                                 _P, _I64, _P, _SZ, _P], _I32),
    "hgin_gin_mlp_fwd_zy_bf16": ([_P, _I64, _I64, _P, _I64, _P, _P, _P, _P, _P, _P, _I64, _I64, _I64, _P], _I32),
    "hgin_gin_mlp_bwd_w_zy_bf16": ([_P, _I64, _P, _P, _P, _P, _I64, _I64, _P, _I64, _I64, _I64, _I64, _P, _I64, _P,
                                    _P, _P, _I64, _P, _SZ, _P], _I32),
    "hgin_self_wgrad_workspace_size": ([_I64, _I64, ctypes.POINTER(_SZ)], _I32),
    "hgin_self_wgrad_f32": ([_P, _I64, _P, _I64, _I64, _I64, _I64, _I32, _P, _P, _I64, _P, _P, _SZ, _P], _I32),
    "hgin_combine_bwd_bf16": ([_P, _I64, _P, _I64, _I64, _I64, _P, _P, _I64, _P, _P, _SZ, _P], _I32),
    "hgin_head_mape_workspace_size": ([_I64, _I64, ctypes.POINTER(_SZ)], _I32),
    "hgin_head_mape_fwd_f32": ([_P, _I64, _I64, _I64, _P, _P, _P, _P, _P, _P, _P, _SZ, _P], _I32),
    "hgin_head_mape_fwd_bf16": ([_P, _I64, _I64, _I64, _P, _P, _P, _P, _P, _P, _P, _SZ, _P], _I32),
    "hgin_head_mape_bwd_f32": ([_P, _I64, _I64, _I64, _P, _P, _P, _P, _P, _P, _I64, _P, _P, _P, _SZ, _P], _I32),
    "hgin_head_mape_bwd_bf16": ([_P, _I64, _I64, _I64, _P, _P, _P, _P, _P, _P, _I64, _P, _P, _P, _SZ, _P], _I32),
    "hgin_qt_traffic": ([_P, _I64, _P, _P, _P, _P, _P, _P], _I32),
    "hgin_qt_link_sum": ([_P, _P, _P, _P, _I64, _P, _P], _I32),
    "hgin_qt_links": ([_P, _I64, _P, _P, _P, _I32, _P, _P, _P, _P, _P, _P], _I32),
    "hgin_qt_delay": ([_P, _I64, _P, _P, _P, _P, _P], _I32),
    "hgin_batched_copy": ([_P, _I64, _I64, _P], _I32),
    "hgin_neg_sample": ([_U64, _U64, _I64, _I64, _P, _P], _I32),
    "hgin_dot_decode_fwd_f32": ([_P, _P, _I64, _P, _I64, _P, _I64, _I64, _P, _P], _I32),
    "hgin_dot_decode_bwd_f32": ([_P, _P, _P, _I64, _P, _P, _I64, _I64, _P, _I64, _P], _I32),
    "hgin_aggregate_long_f32": ([_P, _P, _I64, _P, _P, _I64, _P, _I64, _I64, _P, _I64, _I64, _P, _I32, _P, _I64, _P,
                                 _SZ, _P], _I32),
    "hgin_aggregate_long_bf16": ([_P, _P, _I64, _P, _P, _I64, _P, _I64, _I64, _P, _I64, _I64, _P, _I32, _P, _I64, _P,
                                  _SZ, _P], _I32),
    "hgin_nt_planes_size": ([_I64, _I64, _I32, ctypes.POINTER(_SZ)], _I32),
    "hgin_nt_planes_f32": ([_P, _I64, _I64, _I64, _P, _P], _I32),
    "hgin_nt_planes_bf16": ([_P, _I64, _I64, _I64, _P, _P], _I32),
    "hgin_global_pool_workspace_size": ([_I64, _I64, ctypes.POINTER(_SZ)], _I32),
    "hgin_global_pool_f32": ([_P, _I64, _P, _I64, _I64, _P, _I64, _P, _P, _SZ, _P], _I32),
    "hgin_global_pool_bf16": ([_P, _I64, _P, _I64, _I64, _P, _I64, _P, _P, _SZ, _P], _I32),
    "hgin_gat_logits_f32": ([_P, _I64, _I64, _I64, _I64, _P, _P, _P], _I32),
    "hgin_gat_attn_fwd_f32": ([_P, _P, _I64, _I64, _I64, _P, _I64, _P, _P, ctypes.c_float, _P, _P, _I64, _P, _P, _I64,
                               _P], _I32),
    "hgin_gat_attn_supported": ([_I64, _I64], _I32),
    "hgin_gat_fwd_f32": ([_P, _P, _I64, _I64, _I64, _P, _I64, _P, _P, ctypes.c_float, _P, _P, _I64, _P, _P, _I64, _P],
                         _I32),
    "hgin_gat_bwd_dst_f32": ([_P, _P, _I64, _I64, _I64, _P, _I64, _P, _I64, _P, _P, _P, ctypes.c_float, _P, _P, _P,
                              _P, _I64, _P], _I32),
    "hgin_gat_bwd_src_f32": ([_P, _P, _P, _I64, _I64, _I64, _P, _I64, _P, _P, _P, _P, _P, _I64, _P], _I32),
    "hgin_gat_wsum_workspace_size": ([_I64, _I64, _I64, ctypes.POINTER(_SZ)], _I32),
    "hgin_gat_wsum_f32": ([_P, _I64, _I64, _I64, _I64, _P, _P, _P, _SZ, _P], _I32),
    "hgin_sb_args_size": ([], _SZ),
    "hgin_sb_args_offsets": ([_P, _I64], _I32),
    "hgin_sb_readout_lds_bytes": ([_I64, _I64, _I32, _I32, _P, _I32, ctypes.POINTER(_SZ)], _I32),
    "hgin_sb_step": ([_P, _SZ, _SZ, _P], _I32),
    "hgin_host_alloc": ([_SZ, ctypes.POINTER(ctypes.c_void_p)], _I32),
    "hgin_host_free": ([_P], _I32),
    "hgin_trace_enable": ([_I32], _I32),
    "hgin_trace_read": ([ctypes.c_char_p, _SZ], _SZ),
}
ABI_VERSION = 8


def lib() -> ctypes.CDLL:
    """The loaded libhgin.so (built on first use if missing or stale)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        try:
            path = build()
            handle = ctypes.CDLL(path, mode=ctypes.RTLD_LOCAL)
        except (OSError, HginUnavailable) as e:
            raise HginUnavailable(f"libhgin.so unavailable: {e}") from e
        for name, (args, res) in _SIGS.items():
            fn = getattr(handle, name)
            fn.argtypes = args
            fn.restype = res
        if handle.hgin_abi_version() != ABI_VERSION:
            raise HginUnavailable("libhgin.so ABI version mismatch")
        _lib = handle
        return _lib


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = lib().hgin_last_error().decode(errors="replace")
        raise HginError(f"{what} failed with status {rc}: {msg}")


def call(name: str, *args) -> None:
    check(getattr(lib(), name)(*args), name)


class trace_launches:
    """Context manager recording the kernel variant of every libhgin.so launch issued inside it
    (hgin_trace_enable / hgin_trace_read); ``.kernels`` is the list of tags, in launch order."""

    def __enter__(self):
        self.kernels = []
        lib().hgin_trace_enable(1)
        return self

    def __exit__(self, *exc):
        h = lib()
        n = h.hgin_trace_read(None, 0)
        buf = ctypes.create_string_buffer(n + 1)
        h.hgin_trace_read(buf, n + 1)
        h.hgin_trace_enable(0)
        self.kernels = [t for t in buf.value.decode().split("\n") if t]
        return False


def exported_symbols():
    return list(_SIGS.keys())
