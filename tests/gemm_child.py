"""Child process of tests/test_gpu_gemm_switch.py: the bf16 GIN MLP GEMM (hgin_gin_mlp_fwd_bf16) at the shapes
of the weight-stationary kernel (K 128 / 256 / 512, N 128 / 256; ragged M, M below one block, many blocks
per workgroup; accum / z present or not; a two-source A) under the process-static HGIN_* switches its parent
set.  Checks every output against an fp32 evaluation of the same bf16 operands and saves them, so the parent
can compare switch settings bit for bit.

    python tests/gemm_child.py OUT.pt
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (HERE, ROOT, os.path.join(ROOT, "gnn-link-prediction_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402

from hgin import ops  # noqa: E402

BF = torch.bfloat16
CASES = [  # (M, K, N, accum, save_z, k1 of a two-source A or 0)
    (300_007, 512, 256, True, True, 0), (1, 512, 256, True, True, 0), (31, 256, 256, False, True, 0),
    (70_001, 256, 256, True, False, 0), (50_000, 128, 256, True, True, 0), (65, 128, 256, False, False, 0),
    (100_003, 512, 128, True, True, 0), (20_000, 256, 128, True, True, 0), (9_999, 128, 128, True, True, 0),
    (40_000, 512, 256, True, True, 256), (12_345, 256, 128, False, True, 128),
]


def run(M, K, N, with_acc, save_z, k1, g):
    a = torch.randn(M, K, device="cuda", generator=g).to(BF)
    w = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).to(BF)
    b = torch.randn(N, device="cuda", generator=g)
    s = torch.tensor([0.25], device="cuda")
    acc = torch.randn(M, N, device="cuda", generator=g).to(BF) if with_acc else None
    if k1:
        a1, a2 = a[:, :k1].contiguous(), a[:, k1:].contiguous()
        z, y = ops.gin_mlp_fwd(a1, w, b, s, acc, save_z=save_z, comb2=a2)
    else:
        z, y = ops.gin_mlp_fwd(a, w, b, s, acc, save_z=save_z)
    zr = a.float() @ w.float().t() + b
    yr = torch.where(zr > 0, zr, 0.25 * zr) + (acc.float() if with_acc else 0.0)
    tol = lambda r: 2 ** -8 * r.abs() + 1e-3 * (a.float().abs() @ w.float().abs().t() + 1)   # noqa: E731
    assert bool(((y.float() - yr).abs() <= tol(yr)).all()), (M, K, N, "y")
    if save_z:
        assert bool(((z.float() - zr).abs() <= tol(zr)).all()), (M, K, N, "z")
    out = {"y": y.cpu()}
    if save_z:
        out["z"] = z.cpu()
    return out


def main():
    torch.cuda.init()
    g = torch.Generator(device="cuda").manual_seed(7)
    res = {f"{c}": run(*c, g) for c in CASES}
    torch.save(res, sys.argv[1])
    print("gemm child ok", {k: v for k, v in os.environ.items() if k.startswith("HGIN_")}, flush=True)


if __name__ == "__main__":
    main()
