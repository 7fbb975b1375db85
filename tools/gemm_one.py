"""One fp32 GEMM shape, a few launches (a PMC target): python tools/gemm_one.py [fwd|dw] M K N"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gnn-link-prediction_amd")]

import torch  # noqa: E402

from hgin import ops  # noqa: E402


def main():
    kind = sys.argv[1] if len(sys.argv) > 1 else "fwd"
    M, K, N = (int(v) for v in (sys.argv[2:5] if len(sys.argv) > 4 else (3_000_000, 512, 256)))
    g = torch.Generator(device="cuda").manual_seed(1)
    a = torch.randn(M, K, device="cuda", generator=g)
    if kind == "fwd":
        w = torch.randn(N, K, device="cuda", generator=g) / K ** 0.5
        b = torch.randn(N, device="cuda", generator=g)
        s = torch.tensor([0.25], device="cuda")
        fn = lambda: ops.gin_mlp_fwd(a[:, :K // 2], w, b, s, None, comb2=a[:, K // 2:])   # noqa: E731
    else:
        gy = torch.randn(M, N, device="cuda", generator=g)
        z = torch.randn(M, N, device="cuda", generator=g)
        s = torch.tensor([0.25], device="cuda")
        fn = lambda: ops.mlp_bwd_w(gy, z, s, a[:, :K // 2], a[:, K // 2:])   # noqa: E731
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    print("done", kind, M, K, N)


if __name__ == "__main__":
    main()
