"""Child process of tests/test_gpu_h2.py, started with HGIN_F32_GEMM=h2 (process-static): the fp32 NT GEMMs on the
scaled two-term fp16 split (k_gemm_nt_h2) against a float64 evaluation of the same operands.

Operands stress the scaling: rows of very different magnitude (1e-15 .. 1e15), all-zero rows, rows whose first K-tiles
are tiny and later ones huge (the accumulator-rescale path), a weight row far from the others, ragged M and N.
Bound: |c - c64| <= 2^-18 (sum_k |a_k b_k|) elementwise — the two-term split's representation error (~2^-21 per
product) plus the fp32 accumulation over K (tests/gemm_child.py holds the six-product split to 1e-5 of the same sum);
the epilogue outputs carry the bound through bias / PReLU / accum.

    HGIN_F32_GEMM=h2 python tests/h2_child.py
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (HERE, ROOT, os.path.join(ROOT, "gnn-link-prediction_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402

from hgin import _lib, ops  # noqa: E402

TOL = 2.0 ** -18


def operands(M, K, N, g):
    a = torch.randn(M, K, device="cuda", generator=g)
    a[3::11] *= 1e15
    a[5::11] *= 1e-15
    a[7::11] = 0.0
    if K > 64:   # first two K-tiles tiny, the rest large: the row exponent is lowered mid-loop
        a[9::11, :64] *= 1e-6
        a[10::11, 32:] *= 1e5
    w = torch.randn(N, K, device="cuda", generator=g) / K ** 0.5
    w[N // 2] *= 1e10
    w[:, K // 3] *= 1e-12
    return a, w


def check(c, ref, bound, what, extra=0.0):
    bad = (c.double() - ref).abs() > TOL * bound + extra + 1e-300
    assert not bool(bad.any()), (what, int(bad.sum()), float(((c.double() - ref).abs() / bound.clamp_min(1e-300)).max()))
    assert bool(torch.isfinite(c).all()), what


def main():
    assert ops.H2, "start with HGIN_F32_GEMM=h2"
    torch.cuda.init()
    g = torch.Generator(device="cuda").manual_seed(11)
    s = torch.tensor([0.25], device="cuda")
    n_ok = 0
    for M, K, N, k1, eps in [(70_001, 512, 256, 256, 0.37), (40_000, 256, 256, 0, None), (1, 512, 256, 0, None),
                             (999, 256, 128, 128, -0.2), (5_003, 128, 96, 0, None), (3_000, 64, 32, 0, None)]:
        a, w = operands(M, K, N, g)
        b = torch.randn(N, device="cuda", generator=g)
        acc = torch.randn(M, N, device="cuda", generator=g)
        with _lib.trace_launches() as tr:
            if k1:
                e2 = torch.tensor([eps], device="cuda")
                z, y = ops.gin_mlp_fwd(a[:, :k1].contiguous(), w, b, s, acc, comb2=a[:, k1:].contiguous(), eps2=e2)
                a = torch.cat([a[:, :k1], a[:, k1:] * (1.0 + e2)], 1)   # the kernel's self term, fp32 product
            else:
                z, y = ops.gin_mlp_fwd(a, w, b, s, acc)
            torch.cuda.synchronize()
        assert any(k.startswith("k_gemm_nt_h2<EPI1") for k in tr.kernels), tr.kernels
        zr = a.double() @ w.double().t()
        bound = a.double().abs() @ w.double().abs().t()
        zb = zr + b.double()                       # z = fl(c + b): one more rounding
        check(z, zb, bound + b.double().abs(), ("z", M, K, N), 2 ** -23 * zb.abs())
        yr = torch.where(z.double() > 0, z.double(), 0.25 * z.double()) + acc.double()
        assert bool(((y.double() - yr).abs() <= 2 ** -23 * yr.abs() + 1e-300).all()), ("y", M, K, N)
        # plain dX GEMM (EPI 0) and the linear head form (EPI 2)
        with _lib.trace_launches() as tr:
            c = ops.gemm_nt(a, w)
            torch.cuda.synchronize()
        assert any(k.startswith("k_gemm_nt_h2<EPI0") for k in tr.kernels), tr.kernels
        check(c, zr, bound, ("gemm_nt", M, K, N))
        n_ok += 1
    # dX with the self-term backward (EPI 4) at the cfg3 add-layer shape
    M, K, N = 50_001, 256, 256
    a, w = operands(M, K, N, g)
    xd = torch.randn(M, N, device="cuda", generator=g)
    eps = torch.tensor([0.3], device="cuda")
    with _lib.trace_launches() as tr:
        c, gx, ge = ops.gemm_nt_combine(a, w, xd, eps, 0, True)
        torch.cuda.synchronize()
    assert any(k.startswith("k_gemm_nt_h2<EPI4") for k in tr.kernels), tr.kernels
    cr = a.double() @ w.double().t()
    check(c, cr, a.double().abs() @ w.double().abs().t(), "combine c")
    assert torch.equal(gx, (1.0 + eps) * c), "combine g_x_dst"
    ge_ref = float((c.double() * xd.double()).sum())
    assert abs(float(ge) - ge_ref) <= 1e-5 * float((c.double() * xd.double()).abs().sum()), (float(ge), ge_ref)
    print(f"h2 child ok ({n_ok + 1} shapes)", flush=True)


if __name__ == "__main__":
    main()
