"""A/B: the fp32 forward GIN GEMM with A split in the kernel (default, k_gemm_nt kBdma) vs A pre-split into row
images (hgin_a_planes_f32 + hgin_gin_mlp_fwd_apl_f32, k_gemm_nt kApl): time per launch, the planes pass alone, and
bitwise equality of z / y.   HGIN_APL_OCC=3 python tools/apl_bench.py   (default 2 workgroups per CU)
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gnn-link-prediction_amd")]

import torch  # noqa: E402

from hgin import _lib, ops  # noqa: E402
from hgin.ops import _p, _stream  # noqa: E402


def timeit(fn, reps=10):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    h = _lib.lib()
    P, I64 = ctypes.c_void_p, ctypes.c_int64
    h.hgin_a_planes_f32.argtypes = [P, I64, I64, I64, P, P]
    h.hgin_gin_mlp_fwd_apl_f32.argtypes = [P, P, P, P, P, P, P, I64, I64, I64, P]
    g = torch.Generator(device="cuda").manual_seed(5)
    for M, K, N, with_acc in [(6_000_000, 512, 256, True), (3_000_000, 512, 256, False), (6_000_000, 256, 256, True)]:
        a = torch.randn(M, K, device="cuda", generator=g)
        w = torch.randn(N, K, device="cuda", generator=g) / K ** 0.5
        b = torch.randn(N, device="cuda", generator=g)
        s = torch.tensor([0.25], device="cuda")
        acc = torch.randn(M, N, device="cuda", generator=g) if with_acc else None
        wp = ops.nt_planes(w)
        ap = torch.empty(M * K * 6, dtype=torch.uint8, device="cuda")
        mk = lambda: _lib.call("hgin_a_planes_f32", _p(a), a.stride(0), M, K, _p(ap), _stream(a))  # noqa: E731
        z1, y1 = torch.empty(M, N, device="cuda"), torch.empty(M, N, device="cuda")

        def apl():
            _lib.call("hgin_gin_mlp_fwd_apl_f32", _p(ap), _p(wp), _p(b), _p(s), _p(acc), _p(z1), _p(y1), M, N, K,
                      _stream(a))

        base = lambda: ops.gin_mlp_fwd(a, w, b, s, acc)  # noqa: E731
        z0, y0 = base()
        mk()
        with _lib.trace_launches() as tr:
            apl()
        torch.cuda.synchronize()
        same = torch.equal(z0, z1) and torch.equal(y0, y1)
        t0, tp, t1 = timeit(base), timeit(mk), timeit(apl)
        gb = 4 * (M * K + M * N * (2 + (acc is not None))) / 1e9
        gb_apl = gb + 2 * M * K / 1e9
        print(f"M={M} K={K} N={N} acc={with_acc}: split-in-kernel {t0:7.3f} ms ({gb / t0:5.2f} TB/s) | "
              f"planes pass {tp:7.3f} ms | pre-split GEMM {t1:7.3f} ms ({gb_apl / t1:5.2f} TB/s) | bitwise {same} | "
              f"{sorted(set(tr.kernels))} occ={os.environ.get('HGIN_APL_OCC', '2')}", flush=True)
        del a, w, acc, ap, z0, y0, z1, y1
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
