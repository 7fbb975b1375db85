"""GPU parity of every libhgin.so kernel against the CPU oracle (bit-exact for index and sequential-sum
work; stated tolerances for the MFMA GEMM and the decoder's reduction)."""
import re

import numpy as np
import pytest
import torch

from hgin import _lib, ops
from oracle import c_oracle as co
from oracle.pyg_cpu import propagate_sum

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rand_graph(E, n_src, n_dst, seed, zipf=False):
    rng = np.random.default_rng(seed)
    src = rng.integers(0, n_src, E)
    if zipf and n_dst > 0:
        dst = np.minimum(rng.zipf(1.1, E) - 1, n_dst - 1)
    else:
        dst = rng.integers(0, max(n_dst, 1), E)
    return np.stack([src, dst]).astype(np.int64)


# ------------------------------------------------------------------------------------------ A12 CSR
@pytest.mark.parametrize("E,n_src,n_dst", [(0, 4, 6), (1, 1, 1), (5, 3, 1), (1000, 50, 37), (4096, 10, 300),
                                           (4097, 300, 10), (70000, 5000, 2000), (200000, 100, 70000)])
@pytest.mark.parametrize("key_row", [1, 0])
def test_csr_build_bit_exact(E, n_src, n_dst, key_row):
    ei = _rand_graph(E, n_src, n_dst, seed=E + key_row)
    n_rows, n_cols = (n_dst, n_src) if key_row == 1 else (n_src, n_dst)
    ref_rowptr, ref_col, ref_perm, st = co.csr_build(ei, key_row, n_rows, n_cols)
    assert st == 0
    csr = ops.build_csr(torch.from_numpy(ei).to(DEV), key_row, n_rows, n_cols)
    assert np.array_equal(csr.rowptr.cpu().numpy(), ref_rowptr)
    assert np.array_equal(csr.col.cpu().numpy(), ref_col)
    assert np.array_equal(csr.perm.cpu().numpy(), ref_perm)


def test_csr_build_skewed_and_large():
    ei = _rand_graph(1_000_000, 600_000, 300_000, seed=11, zipf=True)
    ref = co.csr_build(ei, 1, 300_000, 600_000)
    csr = ops.build_csr(torch.from_numpy(ei).to(DEV), 1, 300_000, 600_000)
    assert np.array_equal(csr.rowptr.cpu().numpy(), ref[0])
    assert np.array_equal(csr.col.cpu().numpy(), ref[1])


def test_csr_build_full_size_properties():
    """cfg2's largest relation (3M edges): round trip against a stable device sort (size-independent)."""
    g = torch.Generator(device=DEV).manual_seed(0)
    E, n_src, n_dst = 3_000_000, 600_000, 300_000
    ei = torch.stack([torch.randint(0, n_src, (E,), device=DEV, generator=g),
                      torch.randint(0, n_dst, (E,), device=DEV, generator=g)])
    csr = ops.build_csr(ei, 1, n_dst, n_src)
    order = torch.sort(ei[1], stable=True).indices
    assert torch.equal(csr.perm.long(), order)
    assert torch.equal(csr.col.long(), ei[0][order])
    deg = torch.bincount(ei[1], minlength=n_dst)
    assert torch.equal(csr.rowptr[1:].long() - csr.rowptr[:-1].long(), deg)
    assert int(csr.rowptr[-1]) == E


def test_csr_out_of_range_raises():
    ei = torch.tensor([[0, 1, 2], [0, 5, 1]], device=DEV)
    with pytest.raises(IndexError, match="dst index out of range"):
        ops.build_csr(ei, 1, 3, 3)
    ei = torch.tensor([[0, 7, 2], [0, 1, 1]], device=DEV)
    with pytest.raises(IndexError, match="src index out of range"):
        ops.build_csr(ei, 1, 3, 3)
    ei = torch.tensor([[0, -1], [0, 1]], device=DEV)
    with pytest.raises(IndexError):
        ops.build_csr(ei, 1, 3, 3)


# ----------------------------------------------------------------------------------- A3/A4 aggregate
@pytest.mark.parametrize("F_src,F_dst", [(1, 1), (3, 3), (4, 4), (3, 7), (8, 8), (12, 4), (16, 16), (64, 64),
                                         (128, 128), (256, 256), (260, 260), (128, 3)])
@pytest.mark.parametrize("mode", [0, 1, 2])
def test_aggregate_bit_exact(F_src, F_dst, mode):
    if mode == 1 and F_src != F_dst:
        pytest.skip("add needs equal widths")
    E, n_src, n_dst = 9000, 700, 500
    ei = _rand_graph(E, n_src, n_dst, seed=F_src * 7 + mode)
    ei[1, :40] = 3            # a high-degree row
    rng = np.random.default_rng(F_src)
    x = rng.standard_normal((n_src, F_src)).astype(np.float32)
    xd = rng.standard_normal((n_dst, F_dst)).astype(np.float32)
    eps = np.float32(-0.171875)
    rowptr, col, _, _ = co.csr_build(ei, 1, n_dst, n_src)
    ref = co.aggregate(rowptr, col, x, xd if mode else None, float(eps), mode)
    csr = ops.build_csr(torch.from_numpy(ei).to(DEV), 1, n_dst, n_src)
    width = F_src + (F_dst if mode == 2 else 0)
    out = torch.full((n_dst, width), float("nan"), device=DEV)
    ops.aggregate_into(csr, torch.from_numpy(x).to(DEV), torch.from_numpy(xd).to(DEV) if mode else None,
                       torch.tensor([eps], device=DEV) if mode else None, mode, out)
    assert np.array_equal(out.cpu().numpy(), ref)


@pytest.mark.parametrize("F,dtype", [(128, torch.float32), (16, torch.float32), (256, torch.float32),
                                     (256, torch.bfloat16), (64, torch.bfloat16)])
@pytest.mark.parametrize("mode", [0, 1, 2])
def test_aggregate_bit_exact_skewed_rows(F, dtype, mode):
    """Zipf(1.1) destinations (rows of 0 .. thousands of edges: col chunks reloaded past one lane group,
    long runs of empty rows) and a uniform tail; more rows than one persistent round of lane groups."""
    n_src, n_dst = 3000, 40000
    zipf = _rand_graph(60000, n_src, n_dst, seed=F + mode, zipf=True)
    unif = _rand_graph(60000, n_src, n_dst, seed=F * 3 + mode)
    ei = np.concatenate([zipf, unif], 1)
    g = torch.Generator().manual_seed(F + 7 * mode)
    x = torch.randn(n_src, F, generator=g).to(dtype)
    xd = torch.randn(n_dst, F, generator=g).to(dtype)
    eps = np.float32(0.3125)
    rowptr, col, _, _ = co.csr_build(ei, 1, n_dst, n_src)
    assert int(np.diff(rowptr).max()) > 1000
    ref = torch.from_numpy(co.aggregate(rowptr, col, x.float().numpy(), xd.float().numpy() if mode else None,
                                        float(eps), mode)).to(dtype)
    # the sequential walk for every row (the long-row split off): bit-exact
    csr = ops.split_long_rows(ops.build_csr(torch.from_numpy(ei).to(DEV), 1, n_dst, n_src), 0)
    assert csr.long is None
    out = torch.full((n_dst, F * (2 if mode == 2 else 1)), float("nan"), device=DEV).to(dtype)
    ops.aggregate_into(csr, x.to(DEV), xd.to(DEV) if mode else None,
                       torch.tensor([eps], device=DEV) if mode else None, mode, out)
    got = out.cpu()
    if dtype == torch.bfloat16:
        assert torch.equal(got.view(torch.int16), ref.view(torch.int16))
    else:
        assert torch.equal(got, ref)


@pytest.mark.parametrize("F,dtype", [(256, torch.float32), (128, torch.float32), (256, torch.bfloat16)])
@pytest.mark.parametrize("mode", [0, 1, 2])
def test_aggregate_long_row_split(F, dtype, mode):
    """Zipf(1.1) destinations with the long-row split on (rows above 256 edges, 128-edge chunks): rows at or
    below the threshold stay bit-exact against the C oracle; split rows are the chunked, re-associated sum —
    within 1e-6 of sum |x| of a float64 evaluation (fp32: chunk and combine adds, ~40 per output) and
    bitwise reproducible; CONCAT's self columns are exact everywhere."""
    n_src, n_dst = 3000, 40000
    ei = np.concatenate([_rand_graph(60000, n_src, n_dst, seed=F + mode, zipf=True),
                         _rand_graph(60000, n_src, n_dst, seed=F * 3 + mode)], 1)
    g = torch.Generator().manual_seed(F + 7 * mode)
    x = torch.randn(n_src, F, generator=g).to(dtype)
    xd = torch.randn(n_dst, F, generator=g).to(dtype)
    eps = np.float32(0.3125)
    rowptr, col, _, _ = co.csr_build(ei, 1, n_dst, n_src)
    deg = np.diff(rowptr)
    ref = torch.from_numpy(co.aggregate(rowptr, col, x.float().numpy(), xd.float().numpy() if mode else None,
                                        float(eps), mode)).to(dtype)
    csr = ops.split_long_rows(ops.build_csr(torch.from_numpy(ei).to(DEV), 1, n_dst, n_src), 256, 128)
    assert csr.long is not None and csr.long.long_rows.numel() == int((deg > 256).sum()) > 3
    outs = []
    for _ in range(2):
        out = torch.full((n_dst, F * (2 if mode == 2 else 1)), float("nan"), device=DEV).to(dtype)
        ops.aggregate_into(csr, x.to(DEV), xd.to(DEV) if mode else None,
                           torch.tensor([eps], device=DEV) if mode else None, mode, out)
        outs.append(out.cpu())
    assert torch.equal(outs[0].view(torch.int16) if dtype == torch.bfloat16 else outs[0],
                       outs[1].view(torch.int16) if dtype == torch.bfloat16 else outs[1])
    got = outs[0]
    short = torch.from_numpy(deg <= 256)
    if dtype == torch.bfloat16:
        assert torch.equal(got[short].view(torch.int16), ref[short].view(torch.int16))
    else:
        assert torch.equal(got[short], ref[short])
    if mode == 2:
        assert torch.equal(got[:, F:].float(), ref[:, F:].float())
    # split rows against float64
    lrows = np.nonzero(deg > 256)[0]
    x64 = x.double().numpy()
    for r in lrows:
        nb = col[rowptr[r]:rowptr[r + 1]]
        want = x64[nb].sum(0)
        if mode == 1:
            want = want + (1.0 + float(eps)) * xd[r].double().numpy()
        scale = np.abs(x64[nb]).sum(0) + (np.abs(xd[r].double().numpy()) * 2 if mode == 1 else 0)
        err = np.abs(got[r, :F].double().numpy() - want)
        tol = (1e-6 * scale + 1e-6) if dtype == torch.float32 else (np.abs(want) * 2 ** -8 + 1e-6 * scale + 1e-6)
        assert (err <= tol).all(), (r, float(err.max()))


def test_aggregate_matches_reference_cpu_op():
    """Against PyG's CPU path itself (index_select + scatter_add_ + cat), bit for bit."""
    g = torch.Generator().manual_seed(5)
    n_src, n_dst, E, F = 3000, 1000, 40000, 128
    ei = torch.stack([torch.randint(0, n_src, (E,), generator=g), torch.randint(0, n_dst, (E,), generator=g)])
    x, xd = torch.randn(n_src, F, generator=g), torch.randn(n_dst, F, generator=g)
    eps = torch.tensor([0.0625])
    ref = torch.cat((propagate_sum(x, ei, n_dst), (1 + eps) * xd), 1)
    graph = ops.relation_graph(ei.to(DEV), n_src, n_dst)
    out = ops.aggregate(x.to(DEV), xd.to(DEV), eps.to(DEV), graph, ops.COMBINE_CONCAT)
    assert torch.equal(out.cpu(), ref)
    ref_add = propagate_sum(x, ei, n_dst)
    ref_add += (1 + eps) * xd
    out = ops.aggregate(x.to(DEV), xd.to(DEV), eps.to(DEV), graph, ops.COMBINE_ADD)
    assert torch.equal(out.cpu(), ref_add)


def test_aggregate_strided_views_and_empty():
    rng = np.random.default_rng(3)
    n_src, n_dst = 50, 40
    ei = _rand_graph(300, n_src, n_dst, seed=9)
    big = torch.from_numpy(rng.standard_normal((n_src, 200)).astype(np.float32)).to(DEV)
    x = big[:, 8:72]                       # ld 200, 16-B aligned start
    x_odd = big[:, 1:65]                   # misaligned start -> scalar path
    csr = ops.build_csr(torch.from_numpy(ei).to(DEV), 1, n_dst, n_src)
    rowptr, col, _, _ = co.csr_build(ei, 1, n_dst, n_src)
    for view in (x, x_odd):
        out = torch.empty(n_dst, 64, device=DEV)
        ops.aggregate_into(csr, view, None, None, 0, out)
        assert np.array_equal(out.cpu().numpy(), co.aggregate(rowptr, col, view.cpu().numpy(), None, 0.0, 0))
    # no edges at all: zeros (+ self term)
    empty = ops.build_csr(torch.zeros(2, 0, dtype=torch.long, device=DEV), 1, n_dst, n_src)
    xd = torch.randn(n_dst, 64, device=DEV)
    out = torch.empty(n_dst, 128, device=DEV)
    ops.aggregate_into(empty, x.contiguous(), xd, torch.tensor([0.5], device=DEV), 2, out)
    assert torch.equal(out[:, :64], torch.zeros(n_dst, 64, device=DEV))
    assert torch.equal(out[:, 64:], 1.5 * xd)


# ------------------------------------------------------------------------------------- A5 MFMA GEMM
@pytest.mark.parametrize("M,N,K", [(1, 1, 1), (37, 8, 6), (1000, 128, 256), (513, 130, 129), (300, 256, 512),
                                   (4096, 128, 128), (65, 3, 1000)])
def test_gin_mlp_fwd(M, N, K):
    g = torch.Generator(device=DEV).manual_seed(M + N + K)
    a = torch.randn(M, K, device=DEV, generator=g)
    w = torch.randn(N, K, device=DEV, generator=g) / K ** 0.5
    b = torch.randn(N, device=DEV, generator=g)
    s = torch.tensor([0.25], device=DEV)
    acc = torch.randn(M, N, device=DEV, generator=g)
    z, y = ops.gin_mlp_fwd(a, w, b, s, acc)
    zr = (a.double() @ w.double().t() + b.double())
    bound = 1e-5 * (a.double().abs() @ w.double().abs().t() + b.double().abs() + 1)
    assert ((z.double() - zr).abs() <= bound).all()
    assert torch.equal(y, acc + torch.where(z > 0, z, s * z))
    _, y2 = ops.gin_mlp_fwd(a, w, b, s, None, save_z=False)
    assert torch.equal(y2, torch.where(z > 0, z, s * z))


def test_gemm_layout_identity_asymmetric():
    """A = I with an asymmetric B must return B^T exactly (catches a transposed C/D map)."""
    K = 64
    a = torch.eye(K, device=DEV)
    b = torch.arange(K * 40, device=DEV, dtype=torch.float32).reshape(40, K)   # [N=40, K]
    c = ops.gemm_nt(a, b)                     # c = a @ b^T = b^T
    assert torch.equal(c, b.t())


@pytest.mark.parametrize("M,N,K1,K2", [(1, 1, 1, 0), (1000, 128, 256, 0), (600, 128, 128, 128), (777, 100, 6, 3),
                                       (50000, 128, 256, 0), (33, 256, 64, 40), (0, 8, 4, 0),
                                       (20011, 32, 128, 0), (5000, 32, 128, 128), (3001, 17, 64, 64)])
def test_gemm_tn(M, N, K1, K2):
    a = torch.randn(M, N, device=DEV)
    b1 = torch.randn(M, K1, device=DEV)
    b2 = torch.randn(M, K2, device=DEV) if K2 else None
    out = ops.gemm_tn(a, b1, b2)
    b = b1 if b2 is None else torch.cat((b1, b2), 1)
    ref = a.double().t() @ b.double()
    assert ((out.double() - ref).abs() <= 1e-5 * (a.double().abs().t() @ b.double().abs() + 1)).all()
    again = ops.gemm_tn(a, b1, b2)
    assert torch.equal(out, again)     # deterministic


def test_linear_prelu_autograd():
    torch.manual_seed(3000)
    x = torch.randn(3000, 256, device=DEV, requires_grad=True)
    lin = torch.nn.Linear(256, 128).to(DEV)
    act = torch.nn.PReLU().to(DEV)
    y = ops.linear_prelu(x, lin.weight, lin.bias, act.weight)
    g = torch.randn_like(y)
    y.backward(g)
    got = [x.grad, lin.weight.grad, lin.bias.grad, act.weight.grad]
    x2 = x.detach().double().requires_grad_()
    l2 = torch.nn.Linear(256, 128).double().to(DEV)
    l2.load_state_dict(lin.state_dict())
    a2 = torch.nn.PReLU().double().to(DEV)
    a2.load_state_dict(act.state_dict())
    z2 = l2(x2)
    y2 = torch.where(y.detach() > 0, z2, a2.weight * z2)   # PReLU branch by the fp32 sign (see below)
    assert torch.allclose(y.double(), y2, rtol=1e-5, atol=1e-5)
    y2.backward(g.double())
    for a, b in zip(got, [x2.grad, l2.weight.grad, l2.bias.grad, a2.weight.grad]):
        assert float((a.double() - b).norm() / b.norm()) < 1e-5


@pytest.mark.parametrize("M,N,K", [(200, 64, 128), (1, 256, 3), (1031, 100, 77)])
def test_gemm_nt(M, N, K):
    a = torch.randn(M, K, device=DEV)
    b = torch.randn(N, K, device=DEV)
    c = ops.gemm_nt(a, b)
    ref = a.double() @ b.double().t()
    assert ((c.double() - ref).abs() <= 1e-5 * (a.double().abs() @ b.double().abs().t() + 1)).all()


# --------------------------------------------------------------------------- A9 backward reductions
@pytest.mark.parametrize("M,N", [(1, 1), (1000, 128), (777, 300), (5, 8)])
def test_prelu_bwd(M, N):
    z = torch.randn(M, N, device=DEV)
    z[0, 0] = 0.0
    gy = torch.randn(M, N, device=DEV)
    a = torch.tensor([0.3], device=DEV)
    g_z, g_a, g_b = ops.prelu_bwd(gy, z, a)
    assert torch.equal(g_z, torch.where(z > 0, gy, a * gy))
    zr = z.double()
    ga_ref = (torch.where(zr > 0, torch.zeros_like(zr), zr) * gy.double()).sum()
    assert abs(float(g_a) - float(ga_ref)) <= 1e-5 * (float((zr * gy.double()).abs().sum()) + 1)
    assert ((g_b.double() - g_z.double().sum(0)).abs() <= 1e-5 * g_z.double().abs().sum(0) + 1e-6).all()
    again = ops.prelu_bwd(gy, z, a)
    assert torch.equal(again[1], g_a) and torch.equal(again[2], g_b)   # deterministic


def test_prelu_bwd_strided_grad():
    """The incoming gradient is often a column slice (cat backward of the readout input)."""
    z = torch.randn(500, 64, device=DEV)
    big = torch.randn(500, 100, device=DEV)
    gy = big[:, 7:71]
    a = torch.tensor([0.2], device=DEV)
    g_z, g_a, g_b = ops.prelu_bwd(gy, z, a)
    assert torch.equal(g_z, torch.where(z > 0, gy, a * gy))


@pytest.mark.parametrize("M,N,K1,K2", [(1000, 128, 256, 0), (600, 128, 128, 128), (50000, 128, 128, 128),
                                       (3000, 128, 128, 128),
                                       (20011, 32, 128, 0), (3001, 17, 64, 64), (777, 100, 6, 3), (5, 8, 4, 4),
                                       (129, 256, 100, 28), (0, 64, 64, 0),
                                       (20011, 256, 256, 0), (3001, 256, 64, 64), (7, 256, 128, 128)])
@pytest.mark.parametrize("want_gz", [False, True])
@pytest.mark.parametrize("strided", [False, True])
def test_mlp_bwd_fused(M, N, K1, K2, want_gz, strided):
    """A9 fused: PReLU + bias backward inside the dW GEMM against a float64 evaluation (the fallback shapes
    and want_gz run the separate passes and return g_z)."""
    big = torch.randn(M, N + 5, device=DEV)
    gy = big[:, 3:3 + N] if strided else big[:, :N].contiguous()   # strided: a column slice (unaligned rows)
    z = torch.randn(M, N, device=DEV)
    if M:
        z[0, 0] = 0.0
    a = torch.tensor([0.3], device=DEV)
    b1 = torch.randn(M, K1, device=DEV)
    b2 = torch.randn(M, K2, device=DEV) if K2 else None
    g_w, g_a, g_b, g_z = ops.mlp_bwd_w(gy, z, a, b1, b2, want_gz=want_gz)
    gz_ref = torch.where(z > 0, gy, a * gy)
    if want_gz or not ops.mlp_bwd_fused(z, N, K1 + K2):
        bad = (g_z != gz_ref).any(1).nonzero().flatten()
        assert bad.numel() == 0, f"g_z rows differ: {bad[:20].tolist()} of {M}"
    else:
        assert g_z is None
    b = b1 if b2 is None else torch.cat((b1, b2), 1)
    gzd = gz_ref.double()
    ref_w = gzd.t() @ b.double()
    assert ((g_w.double() - ref_w).abs() <= 1e-5 * (gzd.abs().t() @ b.double().abs() + 1)).all()
    assert ((g_b.double() - gzd.sum(0)).abs() <= 1e-5 * gzd.abs().sum(0) + 1e-6).all()
    zr = z.double()
    ga_ref = (torch.where(zr > 0, torch.zeros_like(zr), zr) * gy.double()).sum()
    assert abs(float(g_a) - float(ga_ref)) <= 1e-5 * (float((zr * gy.double()).abs().sum()) + 1)
    again = ops.mlp_bwd_w(gy, z, a, b1, b2, want_gz=want_gz)
    assert all(torch.equal(p, q) for p, q in zip(again[:3], (g_w, g_a, g_b)))    # deterministic


def test_mlp_bwd_fused_cfg3_layer0_shape():
    """The largest GEMM of the cfg3 step at its own shape: the first layer's fused PReLU + bias backward + dW
    (N = 256, K = 256 + 256 = [aggregate | x_dst], 1M rows; cfg3 runs it at 3-6M), against float64, with the
    launch trace proving the PReLU backward was folded into the dW (no separate k_rows_bwd<0> pass): by default the
    weight-stationary two-pass form (the PReLU-fused pass over columns [0, 256) storing g_z into a scratch, the plain
    pass over [256, 512))."""
    from hgin import _lib
    M, N, K1, K2 = 1 << 20, 256, 256, 256
    gen = torch.Generator(device=DEV).manual_seed(11)
    gy = torch.randn(M, N, device=DEV, generator=gen)
    z = torch.randn(M, N, device=DEV, generator=gen)
    a = torch.tensor([0.25], device=DEV)
    b1 = torch.randn(M, K1, device=DEV, generator=gen)
    b2 = torch.randn(M, K2, device=DEV, generator=gen)
    with _lib.trace_launches() as tr:
        g_w, g_a, g_b, g_z = ops.mlp_bwd_w(gy, z, a, b1, b2)
    torch.cuda.synchronize()
    assert g_z is None
    want = ((r"k_ws[dp]_f32<256,256,prelu_bwd_fused>", r"k_ws[dp]_f32<256,256>") if ops.DW512_WSD else
            (r"k_gemm_tn_partial<prelu_bwd_fused,split,N256,K512>",))
    assert all(any(re.fullmatch(k, t) for t in tr.kernels) for k in want), tr.kernels
    assert not any(t.startswith("k_rows_bwd<0") for t in tr.kernels)
    zr, gyr = z.double(), gy.double()
    ga_ref = float((torch.where(zr > 0, torch.zeros_like(zr), zr) * gyr).sum())
    assert abs(float(g_a) - ga_ref) <= 1e-5 * (float((zr * gyr).abs().sum()) + 1)
    gzd = torch.where(zr > 0, gyr, 0.25 * gyr)
    del zr, gyr, z, gy
    assert ((g_b.double() - gzd.sum(0)).abs() <= 1e-5 * gzd.abs().sum(0) + 1e-6).all()
    b = torch.cat((b1, b2), 1).double()
    ref_w = gzd.t() @ b
    bound = 1e-5 * (gzd.abs().t() @ b.abs() + 1)
    assert ((g_w.double() - ref_w).abs() <= bound).all()


def test_combine_bwd():
    g = torch.randn(900, 130, device=DEV)
    x = torch.randn(900, 64, device=DEV)
    eps = torch.tensor([0.125], device=DEV)
    gx, ge = ops.combine_bwd(g[:, 66:], x, eps, True)
    assert torch.equal(gx, (1 + eps) * g[:, 66:])
    ref = (g[:, 66:].double() * x.double()).sum()
    assert abs(float(ge) - float(ref)) <= 1e-5 * float((g[:, 66:] * x).abs().sum().double())
    assert torch.equal(ops.combine_bwd(g[:, 66:], x, eps, False)[1], ge)


# ---------------------------------------------------------------------------------- A10 / A11
@pytest.mark.parametrize("seed,offset,n,n_dst", [(0, 0, 1, 1), (1234, 6, 10, 1000), (2**40 + 5, 3, 100003, 300000),
                                                  (7, 2**33 + 1, 4096, 2**31 - 1)])
def test_neg_sample_bit_exact(seed, offset, n, n_dst):
    out = torch.empty(n + 1, dtype=torch.int32, device=DEV)
    from hgin import _lib
    _lib.call("hgin_neg_sample", seed, offset, n, n_dst, ops._p(out[1:]), ops._stream(out))   # unaligned too
    assert np.array_equal(out[1:].cpu().numpy(), co.neg_sample(seed, offset, n, n_dst))


def test_dot_decoder():
    from hgin import linkpred
    rng = np.random.default_rng(1)
    n_src, n_dst, n, F = 300, 200, 5000, 64
    src, dst = rng.integers(0, n_src, n), rng.integers(0, n_dst, n)
    zs = rng.standard_normal((n_src, F)).astype(np.float32)
    zd = rng.standard_normal((n_dst, F)).astype(np.float32)
    ref = co.dot_decode_fwd(src, dst, zs, zd)
    pairs = torch.from_numpy(np.stack([src, dst])).to(DEV)
    zs_t = torch.from_numpy(zs).to(DEV).requires_grad_()
    zd_t = torch.from_numpy(zd).to(DEV).requires_grad_()
    score = linkpred.dot_decode(zs_t, zd_t, pairs)
    assert np.allclose(score.detach().cpu().numpy(), ref, rtol=1e-5, atol=1e-5)
    g = torch.randn(n, device=DEV)
    score.backward(g)
    rp, col, perm, _ = co.csr_build(np.stack([src, dst]), 0, n_src, n_dst)
    assert np.array_equal(zs_t.grad.cpu().numpy(), co.dot_decode_bwd(rp, col, perm, g.cpu().numpy(), zd))
    rp, col, perm, _ = co.csr_build(np.stack([src, dst]), 1, n_dst, n_src)
    assert np.array_equal(zd_t.grad.cpu().numpy(), co.dot_decode_bwd(rp, col, perm, g.cpu().numpy(), zs))


@pytest.mark.parametrize("M,K1,K2,N,act", [(3000, 128, 128, 128, True), (777, 8, 3, 128, True), (2000, 32, 0, 1, False),
                                           (513, 6, 5, 7, False)])
def test_linear_two_source_autograd(M, K1, K2, N, act):
    """The readout's Linear(+PReLU) reading cat((x1, x2)) from two sources, vs a float64 torch reference.
    The reference's PReLU branch follows the sign of the fp32 pre-activation (sign(y) = sign(z) for a > 0):
    float64 and fp32 z can disagree in sign within rounding of 0, and each such element flips a gradient row."""
    torch.manual_seed(M + K1 + K2 + N)
    x1 = torch.randn(M, K1, device=DEV, requires_grad=True)
    x2 = torch.randn(M, K2, device=DEV, requires_grad=True) if K2 else None
    lin = torch.nn.Linear(K1 + K2, N).to(DEV)
    a = torch.nn.PReLU().to(DEV) if act else None
    y = ops.linear_prelu(x1, lin.weight, lin.bias, a.weight if act else None, x2=x2)
    g = torch.randn_like(y)
    y.backward(g)
    x = torch.cat((x1, x2), 1) if K2 else x1
    xr = x.detach().double().requires_grad_()
    wr = lin.weight.detach().double().requires_grad_()
    br = lin.bias.detach().double().requires_grad_()
    zr = xr @ wr.t() + br
    if act:
        ar = a.weight.detach().double().requires_grad_()
        yr = torch.where(y.detach() > 0, zr, ar * zr)
    else:
        yr = zr
    assert torch.allclose(y.double(), yr, rtol=1e-5, atol=1e-5)
    yr.backward(g.double())
    gx = torch.cat((x1.grad, x2.grad), 1) if K2 else x1.grad
    pairs = [(gx, xr.grad), (lin.weight.grad, wr.grad), (lin.bias.grad, br.grad)]
    if act:
        pairs.append((a.weight.grad, ar.grad))
    for got, want in pairs:
        assert float((got.double() - want).norm()) <= 1e-5 * float(want.norm()) + 1e-6


@pytest.mark.gpu
@pytest.mark.parametrize("concat", [True, False])
@pytest.mark.parametrize("shape", [(128, 128), (32, 7), (256, 256)])
def test_self_wgrad(concat, shape):
    """hgin_self_wgrad_f32: the first-layer GINConv's self-term weight gradient and eps gradient."""
    from hgin import ops
    N, f = shape
    dev = "cuda"
    gen = torch.Generator().manual_seed(N + f)
    G = torch.randn(N, 2 * f, generator=gen).to(dev)
    W = torch.randn(N, 2 * f if concat else f, generator=gen).to(dev)
    eps = torch.tensor([0.3], device=dev)
    g_w, g_eps = ops.self_wgrad(G, W, f, concat, eps)
    if concat:
        want_w = torch.cat((G[:, :f], (1 + eps) * G[:, f:]), 1)
        want_eps = (W[:, f:].double() * G[:, f:].double()).sum()
    else:
        want_w = G[:, :f]
        want_eps = (W.double() * G[:, f:].double()).sum()
    assert torch.equal(g_w, want_w)
    assert abs(float(g_eps) - float(want_eps)) <= 1e-5 * float((W.abs().double().sum() * G.abs().max()))
    g_w2, g_eps2 = ops.self_wgrad(G, W, f, concat, eps)
    assert torch.equal(g_eps, g_eps2) and torch.equal(g_w, g_w2)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("M,F,N", [(1000, 128, 128), (777, 48, 40), (5000, 256, 256)])
def test_mlp_fwd_self_term_in_loads(dtype, M, F, N):
    """The concat GINConv forward without the materialised concat: [agg | (1+eps) x_dst] formed in the GEMM's
    tile loads gives bit-for-bit the z / y of the GEMM over the aggregate kernel's concat output."""
    from hgin import ops
    dev = "cuda"
    gen = torch.Generator().manual_seed(M + F + N)
    agg = torch.randn(M, F, generator=gen).to(dev, dtype)
    xd = torch.randn(M, F, generator=gen).to(dev, dtype)
    w = (torch.randn(N, 2 * F, generator=gen) / (2 * F) ** 0.5).to(dev, dtype)
    b = torch.randn(N, generator=gen).to(dev)
    a = torch.tensor([0.25], device=dev)
    eps = torch.tensor([0.37], device=dev)
    self_half = (xd.float() * (1 + eps)).to(dtype)       # the aggregate epilogue's (1+eps)*x_dst, one rounding
    comb = torch.cat((agg, self_half), 1)
    z0, y0 = ops.gin_mlp_fwd(comb, w, b, a, None)
    z1, y1 = ops.gin_mlp_fwd(agg, w, b, a, None, comb2=xd, eps2=eps)
    assert torch.equal(z0, z1) and torch.equal(y0, y1)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("M,K,F_src,F_dst", [(1000, 128, 0, 128), (777, 64, 48, 40), (30000, 128, 128, 128),
                                             (5, 32, 8, 20), (200, 16, 0, 30)])
@pytest.mark.parametrize("want_gx", [True, False])
def test_gemm_nt_combine(dtype, M, K, F_src, F_dst, want_gx):
    """dX GEMM with the fused self-term backward: c equals the plain NT GEMM bit for bit; g_x_dst equals
    hgin_combine_bwd_* on that c bit for bit; g_eps within fp32 reduction-order tolerance."""
    from hgin import ops
    dev = "cuda"
    gen = torch.Generator().manual_seed(M + K + F_dst)
    N = F_src + F_dst
    a = torch.randn(M, K, generator=gen).to(dev, dtype)
    b = torch.randn(N, K, generator=gen).to(dev, dtype)
    xd = torch.randn(M, F_dst, generator=gen).to(dev, dtype)
    eps = torch.tensor([0.2], device=dev)
    c, gx, ge = ops.gemm_nt_combine(a, b, xd, eps, F_src, want_gx)
    c0 = ops.gemm_nt(a, b)
    assert torch.equal(c, c0)
    gx0, ge0 = ops.combine_bwd(c0[:, F_src:], xd, eps, True)
    if want_gx:
        assert torch.equal(gx, gx0)
    else:
        assert gx is None
    ref = (c0[:, F_src:].double() * xd.double()).sum()
    bound = 1e-5 * float((c0[:, F_src:].double() * xd.double()).abs().sum()) + 1e-6
    assert abs(float(ge) - float(ref)) <= bound and abs(float(ge0) - float(ref)) <= bound


@pytest.mark.parametrize("F", [1, 4, 7, 300])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_global_pool_vs_cpu_scatter(F, dtype):
    """hgin_global_pool_*: [mean | max] of every graph's rows broadcast to its rows (models.py:347-352); the mean
    bit-identical to CPU scatter_reduce "mean" (sequential sum, one division), the max exact; graph ids that skip
    values, one-row graphs, a graph longer than a 256-row window, NaN propagation in the max."""
    g = torch.Generator().manual_seed(F)
    sizes = [1, 5, 700, 3, 1, 40, 257]
    ids = [0, 1, 3, 4, 9, 10, 11]                       # 2, 5-8 have no rows
    batch = torch.cat([torch.full((n,), i, dtype=torch.long) for n, i in zip(sizes, ids)])
    x = torch.randn(batch.numel(), F + 3, generator=g)[:, 1:1 + F].to(dtype)    # strided rows
    x[10, 0] = float("nan")                             # graph 3 (rows 6..705): its max / mean are NaN in column 0
    xf = x.float()
    size = int(batch.max()) + 1
    idx = batch.view(-1, 1).expand(-1, F)
    mean = torch.zeros(size, F).scatter_reduce(0, idx, xf, reduce="mean", include_self=False)
    mx = torch.zeros(size, F).scatter_reduce(0, idx, xf, reduce="amax", include_self=False)
    want = torch.cat([mean[batch], mx[batch]], 1).to(dtype)
    with _lib.trace_launches() as tr:
        got = ops.global_pool(x.to(DEV), batch.to(DEV)).cpu()
    assert any(t.startswith("k_seg_pool") for t in tr.kernels)
    assert torch.equal(got.isnan(), want.isnan())
    ok = got.isnan() | (got == want)
    assert bool(ok.all()), (~ok).nonzero()[:10]


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_global_pool_long_segments(dtype):
    """GLOBAL_FEATS on big graphs (one graph of millions of path rows must not be one workgroup's serial
    walk): segments longer than 4096 rows go through 2048-row chunk partials added in chunk order — deterministic, the
    mean within fp32 rounding of a float64 evaluation, the max exact; short segments beside them stay bit-identical
    to CPU scatter mean; a single-graph batch of 1M rows; a NaN inside a long segment propagates."""
    g = torch.Generator().manual_seed(3)
    F = 5
    for sizes in ([1_000_000], [3, 4096, 4097, 10, 9000, 2047, 2049, 1, 6000]):
        batch = torch.cat([torch.full((n,), i, dtype=torch.long) for i, n in enumerate(sizes)])
        x = torch.randn(batch.numel(), F, generator=g).to(dtype)
        if len(sizes) > 1:
            x[4200, 2] = float("nan")                     # inside the 4097-row graph
        xf = x.double()
        size = len(sizes)
        idx = batch.view(-1, 1).expand(-1, F)
        mean = torch.zeros(size, F, dtype=torch.float64).index_add_(0, batch, xf) / torch.tensor(sizes).view(-1, 1)
        mx = torch.zeros(size, F, dtype=torch.float64).scatter_reduce(0, idx, xf, reduce="amax", include_self=False)
        absm = torch.zeros(size, F, dtype=torch.float64).index_add_(0, batch, xf.abs()) / torch.tensor(sizes).view(-1, 1)
        got = ops.global_pool(x.to(DEV), batch.to(DEV), check=True)
        got2 = ops.global_pool(x.to(DEV), batch.to(DEV))
        assert torch.equal(got.isnan(), got2.isnan()) and bool((got.isnan() | (got == got2)).all())   # deterministic
        got = got.cpu().double()
        gm, gx = got[:, :F], got[:, F:]
        ulp = 2 ** -7 if dtype == torch.bfloat16 else 2 ** -20
        wm = mean[batch]
        assert torch.equal(gm.isnan(), wm.isnan())
        fin = ~wm.isnan()
        assert bool(((gm - wm).abs()[fin] <= ulp * absm[batch][fin] + 1e-30).all())
        assert torch.equal(gx.isnan(), mx[batch].isnan())
        assert bool((gx == mx[batch.view(-1)]).logical_or(gx.isnan()).all())
        # short graphs (<= 4096 rows): bit-identical to the CPU scatter mean of the stored dtype
        short = torch.tensor([n <= 4096 for n in sizes])[batch]
        cpu = torch.zeros(size, F).scatter_reduce(0, idx, x.float(), reduce="mean", include_self=False)[batch].to(dtype)
        gs = got[short][:, :F].to(torch.float32).to(dtype)
        assert torch.equal(gs.isnan(), cpu[short].isnan()) and bool((gs.isnan() | (gs == cpu[short])).all())


def test_global_pool_unsorted_batch_raises():
    """A batch vector that is not non-decreasing is flagged on the device (HGIN_STATUS_UNSORTED) and raised."""
    batch = torch.tensor([0, 0, 2, 1, 1, 3], dtype=torch.long, device=DEV)
    x = torch.randn(6, 4, device=DEV)
    with pytest.raises(ValueError, match="non-decreasing"):
        ops.global_pool(x, batch, check=True)
    ops.global_pool(x, batch.sort().values, check=True)   # sorted: no error


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("M,N,K1,K2", [(100003, 256, 256, 0), (4099, 256, 128, 0), (33, 256, 256, 0),
                                       (20000, 128, 128, 128), (1, 128, 256, 0),
                                       (30011, 256, 256, 256), (50000, 128, 256, 256), (17, 128, 384, 128),
                                       (60001, 32, 128, 0), (3001, 64, 64, 64)])
def test_wsd_prelu_fused_equals_two_pass(dtype, M, N, K1, K2):
    """The weight-stationary dW with the PReLU backward folded in (k_wsd_*<..., prelu_bwd_fused>, taken whenever g_z
    is wanted at these shapes; K = 512 = the fused pass over columns [0, 256) + a plain pass over [256, 512) on the
    stored g_z): g_z bit-identical to hgin_prelu_bwd_* (the same fp32 arithmetic and rounding), g_w bit-identical to
    the plain weight-stationary dW on that g_z (same M partition, passes and product order), bias / slope gradients
    within 1e-5 of a float64 evaluation (fixed-order sums, another grouping)."""
    from hgin import _lib
    gen = torch.Generator(device=DEV).manual_seed(M + N + K1)
    gy = torch.randn(M, N, device=DEV, generator=gen).to(dtype)
    z = torch.randn(M, N, device=DEV, generator=gen).to(dtype)
    a = torch.tensor([0.3], device=DEV)
    b1 = torch.randn(M, K1, device=DEV, generator=gen).to(dtype)
    b2 = torch.randn(M, K2, device=DEV, generator=gen).to(dtype) if K2 else None
    with _lib.trace_launches() as tr:
        g_w, g_a, g_b, g_z = ops.mlp_bwd_w(gy, z, a, b1, b2, want_gz=True)
    torch.cuda.synchronize()
    fused = [t for t in tr.kernels if "prelu_bwd_fused" in t]
    if N in (128, 256) or dtype == torch.float32:   # bf16 narrow layers keep the separate pass
        assert fused and not any(t.startswith("k_rows_bwd") for t in tr.kernels), tr.kernels
    gz2, _, _ = ops.prelu_bwd(gy, z, a)
    assert torch.equal(g_z, gz2)
    if N in (128, 256):   # the weight-stationary form: the same kernel / partition as the plain dW on g_z
        assert torch.equal(g_w, ops.gemm_tn(gz2, b1, b2))
    else:                 # the tiled fused kernel: its own split of M; against float64
        b = b1 if b2 is None else torch.cat((b1, b2), 1)
        gzd = gz2.double()
        ref_w = gzd.t() @ b.double()
        assert ((g_w.double() - ref_w).abs() <= 1e-5 * (gzd.abs().t() @ b.double().abs() + 1)).all()
    gzd = torch.where(z.double() > 0, gy.double(), gy.double() * 0.3)
    assert ((g_b.double() - gzd.sum(0)).abs() <= 1e-5 * gzd.abs().sum(0) + 1e-6).all()
    zr = z.double()
    ga_ref = (torch.where(zr > 0, torch.zeros_like(zr), zr) * gy.double()).sum()
    assert abs(float(g_a) - float(ga_ref)) <= 1e-5 * (float((zr * gy.double()).abs().sum()) + 1)
    again = ops.mlp_bwd_w(gy, z, a, b1, b2, want_gz=True)
    assert all(torch.equal(p, q) for p, q in zip(again, (g_w, g_a, g_b, g_z)))
