"""Child process of tests/test_gpu_gemm_switch.py: the bf16 GIN MLP GEMM (hgin_gin_mlp_fwd_bf16) at the shapes
of the weight-stationary kernel (K 128 / 256 / 512, N 128 / 256; ragged M, M below one block, many blocks
per workgroup; accum / z present or not; a two-source A) under the process-static HGIN_* switches its parent
set, and the fp32 forward GEMM at the shapes of its weight-stationary kernel (k_ws_f32).  Also the dX GEMMs (plain
and combine) and the weight-gradient GEMMs.  Checks every output against an fp32 / fp64 evaluation of the same
operands and saves them, so the parent can compare switch settings.

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
CASES = [  # (M, K, N, accum, save_z, k1 of a two-source A or 0, eps of the second source or None)
    (300_007, 512, 256, True, True, 0), (1, 512, 256, True, True, 0), (31, 256, 256, False, True, 0),
    (70_001, 256, 256, True, False, 0), (50_000, 128, 256, True, True, 0), (65, 128, 256, False, False, 0),
    (100_003, 512, 128, True, True, 0), (20_000, 256, 128, True, True, 0), (9_999, 128, 128, True, True, 0),
    (40_000, 512, 256, True, True, 256), (12_345, 256, 128, False, True, 128),
    (60_001, 512, 256, True, True, 256, 0.37), (5_000, 256, 256, False, True, 64, -0.2),
]


def run(M, K, N, with_acc, save_z, k1, eps=None, *, g):
    a = torch.randn(M, K, device="cuda", generator=g).to(BF)
    w = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).to(BF)
    b = torch.randn(N, device="cuda", generator=g)
    s = torch.tensor([0.25], device="cuda")
    acc = torch.randn(M, N, device="cuda", generator=g).to(BF) if with_acc else None
    if k1:
        a1, a2 = a[:, :k1].contiguous(), a[:, k1:].contiguous()
        e2 = torch.tensor([eps], device="cuda") if eps is not None else None
        z, y = ops.gin_mlp_fwd(a1, w, b, s, acc, save_z=save_z, comb2=a2, eps2=e2)
        if eps is not None:   # the kernels' self term: bf16(fp32(1 + eps) * a2), rounded once
            a = torch.cat([a1, (a2.float() * (1.0 + torch.tensor(eps, dtype=torch.float32))).to(BF)], 1)
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


F32_CASES = [  # (M, K, N, accum, save_z) — fp32 forward (split mode: k_ws_f32 at K = N = 256 by default)
    (300_007, 256, 256, True, True), (1, 256, 256, True, True), (31, 256, 256, False, True),
    (70_001, 256, 256, True, False), (65, 128, 128, False, False), (20_000, 128, 128, True, True),
    (40_000, 512, 256, True, True), (1_025, 256, 256, False, False),
    (200_003, 512, 256, True, True),   # enough row tiles for the 128-row tiles (+ B planes by LDS-DMA / the 128 x 256 tile)
]


def run_f32(M, K, N, with_acc, save_z, *, g):
    a = torch.randn(M, K, device="cuda", generator=g)
    w = torch.randn(N, K, device="cuda", generator=g) / K ** 0.5
    b = torch.randn(N, device="cuda", generator=g)
    s = torch.tensor([0.25], device="cuda")
    acc = torch.randn(M, N, device="cuda", generator=g) if with_acc else None
    z, y = ops.gin_mlp_fwd(a, w, b, s, acc, save_z=save_z)
    zr = a.double() @ w.double().t() + b.double()
    yr = torch.where(zr > 0, zr, 0.25 * zr) + (acc.double() if with_acc else 0.0)
    tol = lambda r: 1e-6 * r.abs() + 1e-5 * (a.double().abs() @ w.double().abs().t() + 1)   # noqa: E731
    assert bool(((y.double() - yr).abs() <= tol(yr)).all()), (M, K, N, "y")
    out = {"y": y.cpu()}
    if save_z:
        assert bool(((z.double() - zr).abs() <= tol(zr)).all()), (M, K, N, "z")
        out["z"] = z.cpu()
    return out


F32_CONCAT_CASES = [  # (M, accum, save_z, eps, strided x_dst) — the first layer's fp32 forward [agg | (1 + eps) x_dst] W^T,
    # K = 256 + 256, N = 256: two k_wss_f32 passes by default without accum (round 6), the tiled K = 512 kernel otherwise
    (300_007, False, True, 0.37, False), (1, False, True, 0.37, False), (31, False, False, -0.2, False),
    (70_001, False, True, 0.37, True), (100_003, True, True, 0.37, False), (5_000, False, False, 0.0, True),
]


def run_f32_concat(M, with_acc, save_z, eps, strided, *, g):
    a1 = torch.randn(M, 256, device="cuda", generator=g)
    xd = torch.randn(M, 384 if strided else 256, device="cuda", generator=g)[:, :256]
    w = torch.randn(256, 512, device="cuda", generator=g) / 512 ** 0.5
    b = torch.randn(256, device="cuda", generator=g)
    s = torch.tensor([0.25], device="cuda")
    e2 = torch.tensor([eps], device="cuda")
    acc = torch.randn(M, 256, device="cuda", generator=g) if with_acc else None
    from hgin import _lib
    with _lib.trace_launches() as tr:
        z, y = ops.gin_mlp_fwd(a1, w, b, s, acc, save_z=save_z, comb2=xd, eps2=e2)
    if os.environ.get("HGIN_NT_WS32", "1") != "0" and not with_acc:   # the default takes the two-pass form
        assert any(k.startswith("k_wss_f32<EPI5") for k in tr.kernels) and \
            any(k.startswith("k_wss_f32<EPI1") and k.endswith(",init>") for k in tr.kernels), tr.kernels
    sc = float(torch.tensor(1.0) + torch.tensor(eps))          # fl(1 + eps), as the kernels form it
    a = torch.cat((a1.double(), (torch.tensor(sc) * xd.cpu()).to(xd.device).double()), 1)
    zr = a @ w.double().t() + b.double()
    yr = torch.where(zr > 0, zr, 0.25 * zr) + (acc.double() if with_acc else 0.0)
    tol = lambda r: 1e-6 * r.abs() + 1e-5 * (a.abs() @ w.double().abs().t() + 1)   # noqa: E731
    assert bool(((y.double() - yr).abs() <= tol(yr)).all()), (M, "concat y")
    out = {"y": y.cpu()}
    if save_z:
        assert bool(((z.double() - zr).abs() <= tol(zr)).all()), (M, "concat z")
        out["z"] = z.cpu()
    return out


DX_CASES = [  # (M, K, N, combine: None | (want_gx, with g_prev))  — the backward dX GEMMs (EPI 0 / 4)
    (200_003, 256, 256, None), (31, 512, 256, None), (70_000, 256, 128, None),
    (150_001, 256, 256, (True, True)), (99_999, 256, 256, (True, False)), (40_000, 256, 256, (False, False)),
    (33, 256, 128, (True, True)),
]


def run_dx(M, K, N, comb, *, g):
    """c = a @ b^T (ops.gemm_nt) or the combine form (ops.gemm_nt_combine, self term on every column)."""
    a = torch.randn(M, K, device="cuda", generator=g).to(BF)
    b = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).to(BF)
    cr = a.float() @ b.float().t()
    bound = 2 ** -8 * cr.abs() + 1e-3 * (a.float().abs() @ b.float().abs().t() + 1)
    if comb is None:
        c = ops.gemm_nt(a, b)
        assert bool(((c.float() - cr).abs() <= bound).all()), (M, K, N)
        return {"c": c.cpu()}
    want_gx, with_prev = comb
    xd = torch.randn(M, N, device="cuda", generator=g).to(BF)
    eps = torch.tensor([0.3], device="cuda")
    prev = torch.randn(M, N, device="cuda", generator=g).to(BF) if with_prev else None
    prev0 = prev.clone() if with_prev else None
    c, gx, ge = ops.gemm_nt_combine(a, b, xd, eps, 0, want_gx, g_prev=prev)
    assert bool(((c.float() - cr).abs() <= bound).all()), (M, K, N, "c")
    c32 = c.float()
    ge_ref = float((c32.double() * xd.double()).sum())
    assert abs(float(ge) - ge_ref) <= 1e-5 * float((c32.double() * xd.double()).abs().sum()), (M, float(ge), ge_ref)
    out = {"c": c.cpu(), "tol_g_eps": ge.detach().reshape(1).cpu()}
    if want_gx:
        gr = (torch.tensor(1.3, dtype=torch.float32) * c32).to(BF).float()   # fp32 (1 + eps) * c, rounded once
        if with_prev:
            gr = (prev0.float() + (1.3 * c32)).to(BF).float()
        assert bool(((gx.float() - gr).abs() <= 2 ** -7 * gr.abs() + 1e-6).all()), (M, "g_x_dst")
        out["gx"] = gx.cpu()
    return out


DX_F32_CASES = [  # (M, want_gx, with g_prev) — the fp32 dX GEMM with the self-term backward, K = N = 256
    (150_001, True, True), (99_999, True, False), (40_000, False, False), (33, True, True),
]


def run_dx_f32(M, want_gx, with_prev, *, g):
    """fp32 ops.gemm_nt_combine (k_ws_f32 EPI 4 by default): c within the fp32 bound of an fp64 evaluation,
    g_x_dst exactly fp32((1 + eps) c) [+ g_prev] on the kernel's own c, the eps gradient within 1e-5."""
    K = N = 256
    a = torch.randn(M, K, device="cuda", generator=g)
    b = torch.randn(N, K, device="cuda", generator=g) / K ** 0.5
    xd = torch.randn(M, N, device="cuda", generator=g)
    eps = torch.tensor([0.3], device="cuda")
    prev = torch.randn(M, N, device="cuda", generator=g) if with_prev else None
    prev0 = prev.clone() if with_prev else None
    c, gx, ge = ops.gemm_nt_combine(a, b, xd, eps, 0, want_gx, g_prev=prev)
    cr = a.double() @ b.double().t()
    assert bool(((c.double() - cr).abs() <= 1e-6 * cr.abs() + 1e-5 * (a.double().abs() @ b.double().abs().t())
                 ).all()), (M, "c")
    ge_ref = float((c.double() * xd.double()).sum())
    assert abs(float(ge) - ge_ref) <= 1e-5 * float((c.double() * xd.double()).abs().sum()), (M, float(ge), ge_ref)
    out = {"c": c.cpu(), "tol_g_eps": ge.detach().reshape(1).cpu()}
    if want_gx:
        gr = (1.0 + eps) * c                      # fp32 (1 + eps), then the product, as the epilogue rounds them
        if with_prev:
            gr = prev0 + gr
        assert torch.equal(gx, gr), (M, "g_x_dst")
        out["gx"] = gx.cpu()
    return out


DX_F32_PLAIN_CASES = [  # (M, K, strided a) — the plain fp32 dX GEMM at N = 256 (k_wss_f32 EPI 5 by default, round 6)
    (200_003, 128, False), (31, 128, False), (1, 128, True), (70_001, 256, False), (33_333, 128, True),
]


def run_dx_f32_plain(M, K, strided, *, g):
    """fp32 ops.gemm_nt, N = 256: c within the fp32 bound of an fp64 evaluation (the readout's dX through its
    Linear(512, 128) is K = 128)."""
    N = 256
    a = torch.randn(M, K + (64 if strided else 0), device="cuda", generator=g)[:, :K]
    b = torch.randn(N, K, device="cuda", generator=g) / K ** 0.5
    from hgin import _lib
    with _lib.trace_launches() as tr:
        c = ops.gemm_nt(a, b)
    if os.environ.get("HGIN_NT_WS32", "1") != "0":
        assert any(k.startswith("k_wss_f32<EPI5") for k in tr.kernels), tr.kernels
    cr = a.double() @ b.double().t()
    assert bool(((c.double() - cr).abs() <= 1e-6 * cr.abs() + 1e-5 * (a.double().abs() @ b.double().abs().t())
                 ).all()), (M, K, "c")
    return {"c": c.cpu()}


DW_CASES = [  # (M, N, K, k1 of a two-source B or 0) — the bf16 weight-gradient GEMM (ops.gemm_tn)
    (300_007, 256, 256, 0), (1, 256, 256, 0), (45, 256, 128, 0), (100_000, 128, 256, 128), (77_777, 128, 128, 0),
    (64_001, 256, 256, 256), (200_003, 256, 512, 256), (9_000, 128, 512, 200), (5, 256, 512, 0),
    # fp32 (split mode: k_wsd_f32 by default)
    (300_001, 256, 256, 0, torch.float32), (17, 256, 128, 0, torch.float32), (80_000, 128, 256, 128, torch.float32),
    (60_000, 256, 512, 256, torch.float32), (4_001, 128, 128, 0, torch.float32),
]


def run_dw(M, N, K, k1, dt=BF, *, g):
    a = torch.randn(M, N, device="cuda", generator=g).to(dt)
    b = torch.randn(M, K, device="cuda", generator=g).to(dt)
    out = ops.gemm_tn(a, b[:, :k1].contiguous(), b[:, k1:].contiguous()) if k1 else ops.gemm_tn(a, b)
    ref = a.double().t() @ b.double()
    bound = 1e-5 * (a.double().abs().t() @ b.double().abs()) + 1e-6
    assert bool(((out.double() - ref).abs() <= bound).all()), (M, N, K)
    return {"tol_dw": out.cpu()}


def main():
    torch.cuda.init()
    g = torch.Generator(device="cuda").manual_seed(7)
    res = {f"{c}": run(*c, g=g) for c in CASES}
    res.update({f"f32{c}": run_f32(*c, g=g) for c in F32_CASES})
    res.update({f"f32cat{c}": run_f32_concat(*c, g=g) for c in F32_CONCAT_CASES})
    res.update({f"dx{c}": run_dx(*c, g=g) for c in DX_CASES})
    res.update({f"dxf32{c}": run_dx_f32(*c, g=g) for c in DX_F32_CASES})
    res.update({f"dxf32p{c}": run_dx_f32_plain(*c, g=g) for c in DX_F32_PLAIN_CASES})
    res.update({f"dw{c}": run_dw(*c, g=g) for c in DW_CASES})
    torch.save(res, sys.argv[1])
    print("gemm child ok", {k: v for k, v in os.environ.items() if k.startswith("HGIN_")}, flush=True)


if __name__ == "__main__":
    main()
