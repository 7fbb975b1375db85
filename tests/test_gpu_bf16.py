"""cfg5 (BASELINE.json configs[4]): bf16 storage + bf16 MFMA with fp32 accumulation, on the GPU.

Checkers: the aggregate is bit-exact against the C oracle run on the fp32-widened inputs followed by torch's
float->bfloat16 rounding (the kernel sums in fp32 and rounds once); GEMMs are checked against float64
products of the same bf16 operands (fp32 accumulation error bound + one bf16 rounding of the output);
elementwise backward kernels are bit-exact; the whole model is a mixed-precision tolerance sweep against
the fp32 oracle (bounds written in the test, measured values in profiles/)."""
import numpy as np
import pytest
import torch

from hgin import HetroGIN, _lib, ops
from oracle import c_oracle as co

pytestmark = pytest.mark.gpu
DEV = "cuda"
BF = torch.bfloat16


def _bf(t):
    return t.to(BF)


def _rand_graph(E, n_src, n_dst, seed):
    rng = np.random.default_rng(seed)
    return np.stack([rng.integers(0, n_src, E), rng.integers(0, n_dst, E)]).astype(np.int64)


# ---------------------------------------------------------------------------------------- aggregate
@pytest.mark.parametrize("F_src,F_dst", [(1, 1), (3, 7), (8, 8), (16, 16), (128, 128), (256, 256), (264, 264),
                                         (128, 3), (12, 4)])
@pytest.mark.parametrize("mode", [0, 1, 2])
def test_aggregate_bf16_bit_exact(F_src, F_dst, mode):
    if mode == 1 and F_src != F_dst:
        pytest.skip("add needs equal widths")
    E, n_src, n_dst = 9000, 700, 500
    ei = _rand_graph(E, n_src, n_dst, seed=F_src * 5 + mode)
    ei[1, :60] = 4
    g = torch.Generator().manual_seed(F_src + F_dst)
    x = _bf(torch.randn(n_src, F_src, generator=g))
    xd = _bf(torch.randn(n_dst, F_dst, generator=g))
    eps = np.float32(0.1875)
    rowptr, col, _, _ = co.csr_build(ei, 1, n_dst, n_src)
    ref32 = co.aggregate(rowptr, col, x.float().numpy(), xd.float().numpy() if mode else None, float(eps), mode)
    ref = torch.from_numpy(ref32).to(BF)
    csr = ops.build_csr(torch.from_numpy(ei).to(DEV), 1, n_dst, n_src)
    width = F_src + (F_dst if mode == 2 else 0)
    out = torch.empty(n_dst, width, dtype=BF, device=DEV)
    ops.aggregate_into(csr, x.to(DEV), xd.to(DEV) if mode else None,
                       torch.tensor([eps], device=DEV) if mode else None, mode, out)
    assert torch.equal(out.cpu().view(torch.int16), ref.view(torch.int16))


def test_aggregate_bf16_autograd_matches_fp32_widened():
    g = torch.Generator().manual_seed(2)
    n_src, n_dst, E, F = 2000, 900, 30000, 128
    ei = torch.stack([torch.randint(0, n_src, (E,), generator=g), torch.randint(0, n_dst, (E,), generator=g)])
    graph = ops.relation_graph(ei.to(DEV), n_src, n_dst)
    x = _bf(torch.randn(n_src, F, generator=g)).to(DEV).requires_grad_()
    xd = _bf(torch.randn(n_dst, F, generator=g)).to(DEV).requires_grad_()
    eps = torch.tensor([0.25], device=DEV, requires_grad=True)
    out = ops.aggregate(x, xd, eps, graph, ops.COMBINE_CONCAT)
    assert out.dtype == BF
    go = _bf(torch.randn(n_dst, 2 * F, generator=g)).to(DEV)
    out.backward(go)
    # backward aggregate over the CSC: bit-exact vs the oracle on widened values, one rounding
    rp, col, _, _ = co.csr_build(ei.numpy(), 0, n_src, n_dst)
    ref_gx = torch.from_numpy(co.aggregate(rp, col, go[:, :F].float().cpu().numpy(), None, 0.0, 0)).to(BF)
    assert torch.equal(x.grad.cpu().view(torch.int16), ref_gx.view(torch.int16))
    assert torch.equal(xd.grad, (1.25 * go[:, F:].float()).to(BF))
    ref_ge = (go[:, F:].double() * xd.detach().double()).sum()
    assert abs(float(eps.grad) - float(ref_ge)) <= 1e-4 * float((go[:, F:].double() * xd.double()).abs().sum())


# -------------------------------------------------------------------------------------------- GEMMs
def _gemm_bound(a, b_t, out_is_bf16):
    """|err| <= fp32-accumulation bound (+ half a bf16 ulp of the result when the output is bf16)."""
    mag = a.double().abs() @ b_t.double().abs()
    return 2e-6 * mag + 1e-6, (2.0 ** -8 if out_is_bf16 else 0.0)


@pytest.mark.parametrize("M,N,K", [(1, 1, 1), (37, 8, 6), (1000, 128, 256), (513, 130, 129), (300, 256, 512),
                                   (4096, 128, 128), (65, 3, 1000), (2000, 32, 128)])
def test_gin_mlp_fwd_bf16(M, N, K):
    g = torch.Generator(device=DEV).manual_seed(M * 3 + N + K)
    a = _bf(torch.randn(M, K, device=DEV, generator=g))
    w = _bf(torch.randn(N, K, device=DEV, generator=g) / K ** 0.5)
    b = torch.randn(N, device=DEV, generator=g)
    s = torch.tensor([0.25], device=DEV)
    acc = _bf(torch.randn(M, N, device=DEV, generator=g))
    z, y = ops.gin_mlp_fwd(a, w, b, s, acc)
    assert z.dtype == BF and y.dtype == BF
    zr = a.double() @ w.double().t() + b.double()
    abs_b, rel = _gemm_bound(a, w.t(), True)
    assert ((z.double() - zr).abs() <= abs_b + rel * zr.abs()).all()
    # the epilogue from the (unrounded) fp32 z: y = bf16(acc + prelu(z)); check against the rounded z within
    # one bf16 step of the sum
    yr = acc.double() + torch.where(zr > 0, zr, 0.25 * zr)
    assert ((y.double() - yr).abs() <= abs_b + 2.0 ** -7 * yr.abs() + 2.0 ** -7 * acc.double().abs()).all()


@pytest.mark.parametrize("M,N,K,with_acc", [(3000, 256, 256, False), (3000, 256, 256, True), (2000, 256, 512, True),
                                            (700, 128, 128, False)])
def test_bf16_epilogue_nan_is_canonical(M, N, K, with_acc):
    """A NaN reaching a bf16 epilogue is stored as torch's canonical 0x7FC0 (c10::BFloat16 rounding), whatever sign
    and payload the fp32 value had: v_cvt_pk_bf16_f32 keeps them, pack_bf2 (hgin_common.h) fixes them up on a branch
    only NaN lanes take.  A row holding +inf and -inf gives inf - inf NaNs (either sign) on the columns whose two
    weights share a sign; every element of the other rows is bit-identical to the same call without the poisoned
    rows."""
    g = torch.Generator(device=DEV).manual_seed(M + K)
    a = _bf(torch.randn(M, K, device=DEV, generator=g))
    w = _bf(torch.randn(N, K, device=DEV, generator=g) / K ** 0.5)
    b = torch.randn(N, device=DEV, generator=g)
    s = torch.tensor([0.25], device=DEV)
    acc = _bf(torch.randn(M, N, device=DEV, generator=g)) if with_acc else None
    z0, y0 = ops.gin_mlp_fwd(a, w, b, s, acc)
    bad = [5, 64, M - 1]
    a[5, 3] = float("nan")
    a[64, 0], a[64, 1] = float("inf"), float("-inf")     # inf - inf where the two weights share a sign
    a[M - 1, K - 1] = -float("nan")
    z, y = ops.gin_mlp_fwd(a, w, b, s, acc)
    for out, ref in ((z, z0), (y, y0)):
        bits = out.view(torch.int16)
        assert bool(out[[5, M - 1]].isnan().all())
        assert bool((out[64].isnan() | out[64].isinf()).all()) and bool(out[64].isnan().any())
        assert bool((bits[out.isnan()] == 0x7FC0).all())
        keep = torch.ones(M, dtype=torch.bool, device=DEV)
        keep[bad] = False
        assert torch.equal(bits[keep], ref.view(torch.int16)[keep])


def test_gemm_bf16_identity_asymmetric():
    K = 64
    a = _bf(torch.eye(K, device=DEV))
    b = _bf(torch.arange(K * 40, device=DEV, dtype=torch.float32).reshape(40, K) % 251)   # exact in bf16
    c = ops.gemm_nt(a, b)
    assert torch.equal(c, b.t())


@pytest.mark.parametrize("M,N,K", [(200, 64, 128), (1, 256, 3), (1031, 100, 77), (5000, 256, 128),
                                   # 32-wide K tiles (K % 64 != 0, K % 32 == 0): the readout's dX through Linear(128, 32)
                                   (60001, 128, 32), (1031, 100, 96), (300, 32, 32)])
def test_gemm_nt_bf16(M, N, K):
    a = _bf(torch.randn(M, K, device=DEV))
    b = _bf(torch.randn(N, K, device=DEV))
    with _lib.trace_launches() as tr:
        c = ops.gemm_nt(a, b)
    assert any(t.endswith(",k32>") for t in tr.kernels) == (K % 64 != 0 and K % 32 == 0 and N > 32), tr.kernels
    assert c.dtype == BF
    ref = a.double() @ b.double().t()
    abs_b, rel = _gemm_bound(a, b.t(), True)
    assert ((c.double() - ref).abs() <= abs_b + rel * ref.abs()).all()


@pytest.mark.parametrize("M,N,K1,K2", [(1, 1, 1, 0), (1000, 128, 256, 0), (600, 128, 128, 128), (777, 100, 6, 3),
                                       (50000, 128, 256, 0), (33, 256, 64, 40), (0, 8, 8, 0), (3001, 130, 72, 56)])
def test_gemm_tn_bf16(M, N, K1, K2):
    a = _bf(torch.randn(M, N, device=DEV))
    b1 = _bf(torch.randn(M, K1, device=DEV))
    b2 = _bf(torch.randn(M, K2, device=DEV)) if K2 else None
    out = ops.gemm_tn(a, b1, b2)
    assert out.dtype == torch.float32
    b = b1 if b2 is None else torch.cat((b1, b2), 1)
    ref = a.double().t() @ b.double()
    assert ((out.double() - ref).abs() <= 1e-5 * (a.double().abs().t() @ b.double().abs()) + 1e-6).all()
    assert torch.equal(out, ops.gemm_tn(a, b1, b2))     # deterministic


def test_gemm_tn_bf16_transpose_map():
    """Integer-valued operands (exact in bf16 and fp32): the in-register 8x8 transpose must be exact."""
    M, N, K = 256, 128, 128
    a = _bf((torch.arange(M * N, device=DEV) % 7 - 3).float().reshape(M, N))
    b = _bf((torch.arange(M * K, device=DEV) % 5 - 2).float().reshape(M, K))
    out = ops.gemm_tn(a, b)
    assert torch.equal(out, (a.float().t() @ b.float()))


# ------------------------------------------------------------------------------ backward elementwise
def test_prelu_bwd_bf16():
    z = _bf(torch.randn(1000, 128, device=DEV))
    gy_big = _bf(torch.randn(1000, 160, device=DEV))
    gy = gy_big[:, 16:144]
    a = torch.tensor([0.3], device=DEV)
    g_z, g_a, g_b = ops.prelu_bwd(gy, z, a)
    gz32 = torch.where(z.float() > 0, gy.float(), a * gy.float())
    assert torch.equal(g_z, gz32.to(BF))
    assert ((g_b.double() - gz32.double().sum(0)).abs() <= 1e-5 * gz32.double().abs().sum(0) + 1e-6).all()
    ga_ref = (torch.where(z.float() > 0, torch.zeros_like(gz32), z.float() * gy.float())).double().sum()
    assert abs(float(g_a) - float(ga_ref)) <= 1e-5 * float((z.double() * gy.double()).abs().sum()) + 1e-6


def test_combine_bwd_bf16():
    g = _bf(torch.randn(900, 136, device=DEV))
    x = _bf(torch.randn(900, 64, device=DEV))
    eps = torch.tensor([0.125], device=DEV)
    gx, ge = ops.combine_bwd(g[:, 72:], x, eps, True)
    assert torch.equal(gx, (1.125 * g[:, 72:].float()).to(BF))
    ref = (g[:, 72:].double() * x.double()).sum()
    assert abs(float(ge) - float(ref)) <= 1e-5 * float((g[:, 72:].double() * x.double()).abs().sum())


def test_linear_prelu_bf16_autograd():
    M, K1, K2 = 3000, 128, 128
    x1 = _bf(torch.randn(M, K1, device=DEV)).requires_grad_()
    x2 = _bf(torch.randn(M, K2, device=DEV)).requires_grad_()
    lin = torch.nn.Linear(K1 + K2, 32).to(DEV)
    act = torch.nn.PReLU().to(DEV)
    head = torch.nn.Linear(32, 1).to(DEV)
    h = ops.linear_prelu(x1, lin.weight, lin.bias, act.weight, x2=x2)
    out = ops.linear_prelu(h, head.weight, head.bias, None)
    assert h.dtype == BF and out.dtype == torch.float32
    out.sum().backward()
    # float64 reference on the same bf16 operand values (weights rounded like the kernels' operand copies)
    xr = torch.cat((x1, x2), 1).detach().double().requires_grad_()
    w1 = lin.weight.detach().to(BF).double().requires_grad_()
    b1 = lin.bias.detach().double().requires_grad_()
    a1 = act.weight.detach().double().requires_grad_()
    z1 = xr @ w1.t() + b1
    hr = torch.where(z1 > 0, z1, a1 * z1)
    w2 = head.weight.detach().to(BF).double().requires_grad_()
    b2 = head.bias.detach().double().requires_grad_()
    outr = hr.to(BF).double() @ w2.t() + b2
    assert float((out.double() - outr).norm() / outr.norm()) < 1e-2
    outr.sum().backward()
    for got, want in [(lin.weight.grad, w1.grad), (lin.bias.grad, b1.grad), (head.weight.grad, w2.grad),
                      (head.bias.grad, b2.grad), (torch.cat((x1.grad, x2.grad), 1), xr.grad)]:
        assert float((got.double() - want).norm()) <= 2e-2 * float(want.norm()) + 1e-6


# ------------------------------------------------------------------------- model: tolerance sweep
def _fixture_bf16_vs_fp32(case):
    from conftest import fixture_inputs, fixture_model_kwargs, fixture_state_dict, load_fixture
    from hgin.train import mape
    fx = load_fixture(case)
    model = HetroGIN(**fixture_model_kwargs(fx))
    model.load_state_dict(fixture_state_dict(fx))
    model = model.to(DEV).train()
    x, ei, batch, y = fixture_inputs(fx, DEV)
    out = model({t: v.to(BF) for t, v in x.items()}, ei, batch)
    lv = mape(out, y.reshape(-1, 1))
    torch.sqrt(lv).backward()
    loss = lv.detach()
    ref_out = fx["out"].double()
    err_out = float((out.detach().cpu().double() - ref_out).norm() / ref_out.norm())
    errs = {}
    for name, p in model.named_parameters():
        key = f"grad.{name}"
        if key in fx and p.grad is not None and float(fx[key].norm()) > 0:
            errs[name] = float((p.grad.cpu().double() - fx[key].double()).norm() / fx[key].double().norm())
    return err_out, errs, float(loss), float(fx["loss_value"])


@pytest.mark.parametrize("case", ["cfg1_L2", "wide_L3", "w128_L2", "w256_L3"])
def test_model_bf16_tolerance_sweep(case):
    """bf16 features/activations vs the fp32 reference fixtures.  Bounds: output rel-L2 <= 3e-2, loss within
    2 %, median parameter-gradient rel-L2 <= 5e-2 (bf16 has an 8-bit mantissa: 2^-9 = 2e-3 per rounding,
    compounded over L layers and the readout)."""
    err_out, errs, loss, ref_loss = _fixture_bf16_vs_fp32(case)
    print(f"\n[bf16 sweep] {case}: out rel-L2 {err_out:.3e}, loss {loss:.6f} vs {ref_loss:.6f}, grad rel-L2 "
          f"median {np.median(list(errs.values())):.3e} max {max(errs.values()):.3e}")
    assert err_out <= 3e-2
    assert abs(loss - ref_loss) <= 2e-2 * abs(ref_loss)
    assert np.median(list(errs.values())) <= 5e-2


def test_model_bf16_full_cfg2_step_runs():
    """cfg2-sized bf16 training step (finite loss, every parameter gets a finite gradient)."""
    from hgin.data import CONFIGS, synthetic_graph
    from hgin.train import train_step
    import dataclasses
    cfg = dataclasses.replace(CONFIGS["cfg2"], feat_dtype="bf16")
    g = synthetic_graph(cfg, seed=0, device=DEV)
    assert g.x["path"].dtype == BF
    torch.manual_seed(1997)
    model = HetroGIN(**cfg.model_kwargs({"link": cfg.f_link, "path": cfg.f_path, "node": cfg.f_node})).to(DEV)
    opt = torch.optim.Adam(model.parameters(), lr=1e-3)
    loss = train_step(model, opt, g)
    assert np.isfinite(float(loss))
    for n, p in model.named_parameters():
        if p.grad is not None:
            assert torch.isfinite(p.grad).all(), n


@pytest.mark.parametrize("M,N,K1,K2", [(3000, 128, 128, 128), (20000, 256, 256, 256), (1001, 64, 40, 24),
                                       (777, 24, 16, 0), (500, 20, 16, 3), (0, 64, 64, 0)])
def test_mlp_bwd_fused_bf16(M, N, K1, K2):
    """hgin_gin_mlp_bwd_w_bf16: g_w bit-identical to hgin_prelu_bwd_bf16's rounded g_z -> hgin_gemm_tn_bf16;
    bias / slope gradients (fixed-order sums of the unrounded fp32 g_z) against float64; deterministic.
    (A variant forming g_z in the transposed-read dW kernel's staging passed this test but ran 1.6x slower
    than the two passes: profiles/r01/s4/mlp_bwd_bf16_fused.txt.)"""
    gen = torch.Generator().manual_seed(M + N + K1)
    gy = torch.randn(M, N, generator=gen).to(DEV, BF)
    z = torch.randn(M, N, generator=gen).to(DEV, BF)
    a = torch.tensor([0.3], device=DEV)
    b1 = torch.randn(M, K1, generator=gen).to(DEV, BF)
    b2 = torch.randn(M, K2, generator=gen).to(DEV, BF) if K2 else None
    g_w, g_a, g_b, _ = ops.mlp_bwd_w(gy, z, a, b1, b2)
    gz2, _, _ = ops.prelu_bwd(gy, z, a)
    assert torch.equal(g_w, ops.gemm_tn(gz2, b1, b2))
    gzd = torch.where(z.double() > 0, gy.double(), gy.double() * 0.3)
    assert ((g_b.double() - gzd.sum(0)).abs() <= 1e-5 * gzd.abs().sum(0) + 1e-6).all()
    zr = z.double()
    ga_ref = (torch.where(zr > 0, torch.zeros_like(zr), zr) * gy.double()).sum()
    assert abs(float(g_a) - float(ga_ref)) <= 1e-5 * (float((zr * gy.double()).abs().sum()) + 1)
    again = ops.mlp_bwd_w(gy, z, a, b1, b2)
    assert all(torch.equal(p, q) for p, q in zip(again[:3], (g_w, g_a, g_b)))


@pytest.mark.parametrize("case", ["cfg1_L2", "w256_L3"])
def test_model_bf16_nonzero_eps_vs_fp32(case):
    """The bf16 first layer folds (1 + eps) into the self half of its weight operand (hgin/ops.py _gin_forward; at
    eps = 0, the reference fixtures' initial value, that is the identity, so the sweep above does not see it).  With
    every eps set to 0.37 the bf16 model against the fp32 model on the same parameters and the same bf16-rounded inputs:
    output rel-L2 <= 3e-2, loss within 2 %, median parameter-gradient rel-L2 <= 5e-2 (the sweep's bounds), and the eps
    gradients (sums of N x K products with cancellation, in bf16 operands) within 1e-1 of the fp32 ones (measured
    1.7e-2 / 4.8e-2, profiles/r03/s20)."""
    from conftest import fixture_inputs, fixture_model_kwargs, fixture_state_dict, load_fixture
    from hgin.train import mape
    fx = load_fixture(case)
    x, ei, batch, y = fixture_inputs(fx, DEV)
    x16 = {t: v.to(BF) for t, v in x.items()}
    res = {}
    for name, xin in (("f32", {t: v.float() for t, v in x16.items()}), ("bf16", x16)):
        model = HetroGIN(**fixture_model_kwargs(fx))
        model.load_state_dict(fixture_state_dict(fx))
        with torch.no_grad():
            for n, p in model.named_parameters():
                if n.endswith(".eps"):
                    p.fill_(0.37)
        model = model.to(DEV).train()
        out = model(xin, ei, batch)
        lv = mape(out, y.reshape(-1, 1))
        torch.sqrt(lv).backward()
        res[name] = (out.detach().double(), float(lv.detach()),
                     {n: p.grad.detach().double() for n, p in model.named_parameters() if p.grad is not None})
    (o32, l32, g32), (o16, l16, g16) = res["f32"], res["bf16"]
    err_out = float((o16 - o32).norm() / o32.norm())
    errs = {n: float((g16[n] - g32[n]).norm() / g32[n].norm()) for n in g32 if float(g32[n].norm()) > 0}
    eps_errs = [v for n, v in errs.items() if n.endswith(".eps")]
    print(f"\n[bf16 eps 0.37] {case}: out rel-L2 {err_out:.3e}, loss {l16:.6f} vs {l32:.6f}, grad rel-L2 median "
          f"{np.median(list(errs.values())):.3e}, eps grads max {max(eps_errs):.3e}")
    assert err_out <= 3e-2 and abs(l16 - l32) <= 2e-2 * abs(l32)
    assert np.median(list(errs.values())) <= 5e-2
    assert eps_errs and max(eps_errs) <= 1e-1


@pytest.mark.parametrize("M,N,K1,K2,slope", [(20000, 256, 256, 0, 0.25), (3000, 128, 128, 0, 0.25),
                                              (5000, 256, 256, 256, 0.25), (4001, 128, 256, 256, 0.3),
                                              (777, 64, 64, 0, 0.25), (9000, 256, 256, 0, -0.1),
                                              (9000, 256, 256, 0, 0.0), (31, 256, 256, 0, 0.25)])
def test_mlp_zy_bf16_matches_plain(M, N, K1, K2, slope):
    """The z-from-y pair (hgin_gin_mlp_fwd_zy_bf16 / hgin_gin_mlp_bwd_w_zy_bf16, ABI 8): y bit-identical to the plain
    forward; g_z, g_w and g_bias bit-identical to the plain backward on the written z (the sign of y is the sign of z
    when the slope is > 0); g_prelu = sum(y g | y <= 0) / slope within the bf16 rounding of z.  With a slope <= 0 the
    forward writes z and everything is bit-identical; N = 64 (no weight-stationary kernel) restores z from y in place
    before the separate PReLU-backward pass."""
    g = torch.Generator(device=DEV).manual_seed(M + N + K1)
    a1 = _bf(torch.randn(M, K1, device=DEV, generator=g))
    a2 = _bf(torch.randn(M, K2, device=DEV, generator=g)) if K2 else None
    w = _bf(torch.randn(N, K1 + K2, device=DEV, generator=g) / (K1 + K2) ** 0.5)
    b = torch.randn(N, device=DEV, generator=g)
    s = torch.tensor([slope], device=DEV)
    z0, y0 = ops.gin_mlp_fwd(a1, w, b, s, None, comb2=a2)
    z1, y1 = ops.gin_mlp_fwd(a1, w, b, s, None, comb2=a2, zy=True)
    assert torch.equal(y1.view(torch.int16), y0.view(torch.int16))
    if slope <= 0:
        assert torch.equal(z1.view(torch.int16), z0.view(torch.int16))
    gy = _bf(torch.randn(M, N, device=DEV, generator=g))
    r0 = ops.mlp_bwd_w(gy, z0, s, a1, a2, want_gz=True)
    r1 = ops.mlp_bwd_w(gy, z1, s, a1, a2, want_gz=True, y_alt=y1)
    assert torch.equal(r1[3].view(torch.int16), r0[3].view(torch.int16))      # g_z
    assert torch.equal(r1[0], r0[0]) and torch.equal(r1[2], r0[2])            # g_w, g_bias
    zd = z0.double()
    bound = 2.0 ** -8 * float((torch.where(zd > 0, 0.0, zd) * gy.double()).abs().sum()) + 1e-6
    assert abs(float(r1[1]) - float(r0[1])) <= bound, (float(r1[1]), float(r0[1]))
    if slope <= 0:
        assert torch.equal(r1[1], r0[1])
