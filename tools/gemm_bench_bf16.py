"""Micro-benchmark of the bf16 (cfg5) MFMA GEMM kernels vs hipBLASLt (torch.mm, bf16) on the shapes of a
cfg2bf / cfg5 step.  These GEMMs are HBM-bound (bf16 MFMA ridge ~300 flop/B), so the figure of merit is
algorithmic bytes / time against the 8 TB/s roofline.  Interleaved rounds, median."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gnn-link-prediction_amd")]

import torch  # noqa: E402

from hgin import ops  # noqa: E402

BF = torch.bfloat16


def timeit(fn, reps=20):
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
    shapes = [(600_000, 256, 128), (300_000, 256, 128), (600_000, 128, 128), (6_000_000, 512, 256),
              (3_000_000, 256, 256)]
    if "--quick" in sys.argv:
        shapes = shapes[:2] + shapes[3:4]
    for M, K, N in shapes:
        a = torch.randn(M, K, device="cuda").to(BF)
        w = (torch.randn(N, K, device="cuda") / K ** 0.5).to(BF)
        b = torch.randn(N, device="cuda")
        s = torch.tensor([0.25], device="cuda")
        acc = torch.randn(M, N, device="cuda").to(BF)
        gz = torch.randn(M, N, device="cuda").to(BF)
        wt = w.t().contiguous()
        cases = [
            ("mlp_fwd(z,y,accum)", lambda: ops.gin_mlp_fwd(a, w, b, s, acc), 2 * (M * K + 3 * M * N)),
            ("mlp_fwd(y only)", lambda: ops.gin_mlp_fwd(a, w, b, s, None, save_z=False), 2 * (M * K + M * N)),
            ("torch.mm a@w^T", lambda: torch.mm(a, w.t()), 2 * (M * K + M * N)),
            ("gemm_tn dW", lambda: ops.gemm_tn(gz, a), 2 * (M * N + M * K)),
            ("torch.mm gz^T@a", lambda: torch.mm(gz.t(), a), 2 * (M * N + M * K)),
            ("gemm_nt dX", lambda: ops.gemm_nt(gz, wt), 2 * (M * N + M * K)),
            ("torch.mm gz@w", lambda: torch.mm(gz, w), 2 * (M * N + M * K)),
        ]
        res = {}
        for _ in range(3):
            for name, fn, _ in cases:
                res.setdefault(name, []).append(timeit(fn))
        print(f"M={M} K={K} N={N}  ({2.0 * M * N * K / 1e9:.1f} GF)")
        for name, _, byts in cases:
            ts = res[name]
            t = sorted(ts)[len(ts) // 2]
            print(f"   {name:22s} {t * 1e3:9.1f} us  {byts / (t / 1e3) / 1e9:7.0f} GB/s  "
                  f"{2.0 * M * N * K / (t / 1e3) / 1e12:6.1f} TF/s")
        del a, w, acc, gz, wt
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
