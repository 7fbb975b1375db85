"""Micro-benchmark of the GIN-update backward on cfg2 / cfg3 shapes: the separate passes (PReLU backward ->
dW TN GEMM [-> dX NT GEMM]) against hgin_gin_mlp_bwd_w (the PReLU backward formed in the dW GEMM's operand
staging).  Interleaved rounds in one process, median.  HGIN_TN_LATEZ is read once per process.
Results: profiles/r01_mlp_bwd_fused.txt."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gnn-link-prediction_amd")]

import torch  # noqa: E402

from hgin import ops  # noqa: E402


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
    shapes = [(600_000, 128, 256), (300_000, 128, 256), (600_000, 128, 128), (1_500_000, 256, 512)]
    if "--cfg5" in sys.argv:   # the first-layer dW-only shapes of a cfg5 step (N = H = 256, K = 2 x 256)
        shapes = [(6_000_000, 256, 512), (3_000_000, 256, 512), (1_000_000, 256, 512)]
    dt = torch.bfloat16 if "--bf16" in sys.argv else torch.float32
    for M, N, K in shapes:
        gy = torch.randn(M, N, device="cuda").to(dt)
        z = torch.randn(M, N, device="cuda").to(dt)
        x = torch.randn(M, K, device="cuda").to(dt)
        w = (torch.randn(N, K, device="cuda") / K ** 0.5).to(dt)
        a = torch.tensor([0.25], device="cuda")

        def separate(dx):
            g_z, g_a, g_b = ops.prelu_bwd(gy, z, a)
            ops.gemm_tn(g_z, x)
            if dx:
                ops.gemm_nt(g_z, w.t().contiguous())

        def fused(dx):
            _, _, _, g_z = ops.mlp_bwd_w(gy, z, a, x, want_gz=dx)
            if dx:
                ops.gemm_nt(g_z, w.t().contiguous())

        res = {}
        for _ in range(3):
            for name, fn in [("prelu_bwd", lambda: ops.prelu_bwd(gy, z, a)),
                             ("gemm_tn", lambda: ops.gemm_tn(gy, x)),
                             ("mlp_bwd_w", lambda: ops.mlp_bwd_w(gy, z, a, x)),
                             ("gemm_nt dX", lambda: ops.gemm_nt(gy, w.t().contiguous())),
                             ("separate dW only", lambda: separate(False)),
                             ("fused dW only", lambda: fused(False)),
                             ("separate dW+dX", lambda: separate(True)),
                             ("fused dW+dX", lambda: fused(True))]:
                res.setdefault(name, []).append(timeit(fn))
        print(f"M={M} N={N} K={K} {dt}  (HGIN_TN_LATEZ={os.environ.get('HGIN_TN_LATEZ', '-')})")
        for name, ts in res.items():
            print(f"   {name:18s} {sorted(ts)[1] * 1e3:9.1f} us")
        del gy, z, x, w
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
