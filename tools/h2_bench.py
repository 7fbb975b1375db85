"""A/B of the fp32 NT GEMMs: six-product bf16 split (default) vs the scaled two-term fp16 split (HGIN_F32_GEMM=h2),
on the cfg3 shapes.  Run once per setting (the switch is process-static); prints time and the error against a
float64 evaluation of 4096 sampled rows, in units of the fp32-evaluation bound sum_k |a_k w_k|.

    HGIN_F32_GEMM=h2 python tools/h2_bench.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gnn-link-prediction_amd")]

import torch  # noqa: E402

from hgin import _lib, ops  # noqa: E402


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
    mode = {k: v for k, v in os.environ.items() if k.startswith("HGIN_")}
    g = torch.Generator(device="cuda").manual_seed(3)
    shapes = [(6_000_000, 512, 256, True, 256), (3_000_000, 512, 256, False, 256), (6_000_000, 256, 256, True, 0),
              (3_000_000, 256, 256, False, 0)]
    for M, K, N, with_acc, k1 in shapes:
        a = torch.randn(M, K, device="cuda", generator=g)
        a[::7] *= 1e3                                  # rows of very different magnitude
        a[1::7] *= 1e-4
        w = torch.randn(N, K, device="cuda", generator=g) / K ** 0.5
        b = torch.randn(N, device="cuda", generator=g)
        s = torch.tensor([0.25], device="cuda")
        acc = torch.randn(M, N, device="cuda", generator=g) if with_acc else None
        if k1:
            a1, a2 = a[:, :k1].contiguous(), a[:, k1:].contiguous()
            fn = lambda: ops.gin_mlp_fwd(a1, w, b, s, acc, comb2=a2)   # noqa: E731
        else:
            fn = lambda: ops.gin_mlp_fwd(a, w, b, s, acc)   # noqa: E731
        with _lib.trace_launches() as tr:
            z, y = fn()
        torch.cuda.synchronize()
        t = timeit(fn)
        rows = torch.randint(0, M, (4096,), device="cuda", generator=g)
        zr = a[rows].double() @ w.double().t() + b.double()
        bound = a[rows].double().abs() @ w.double().abs().t()
        err = ((z[rows].double() - zr).abs() / bound.clamp_min(1e-300)).max().item()
        print(f"M={M} K={K} N={N} acc={with_acc}: {t:8.3f} ms  max |z - z64| / sum|a w| = {err:.3g}  "
              f"kernels {sorted(set(tr.kernels))}  {mode}", flush=True)
        del a, w, acc, z, y
        if k1:
            del a1, a2
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
