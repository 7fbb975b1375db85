"""HetroGAT (models.py:380-506; train.py:120-125 builds it for MODEL == "GAT") on the HIP path, against fixtures made by
executing the reference's own models.py over the shim's PyG 2.0.2 GATConv restatement (tests/golden/make_golden.py
``gat``): config.json exactly (HEADS 16, MP_LAYERS 1, 7/7/3 layout) and a wider 4-head case with the unconvolved
p->n / n->p relations and source / destination index coincidences (GATConv's self-loop removal on bipartite
relations).  Tolerances: attention and aggregates 1e-5 (abs + rel), output and loss 1e-5, gradients 1e-4 of their
norm, the Adam step 1e-5."""
import ctypes

import pytest
import torch

from conftest import fixture_inputs, load_fixture

DEV = "cuda"

pytestmark = pytest.mark.gpu

CASES = ["gat_cfg1_h16", "gat_w16_h4"]


def _kwargs(fx):
    m = fx["meta"]
    ic = {"link": fx["in.x.link"].shape[1], "path": fx["in.x.path"].shape[1], "node": fx["in.x.node"].shape[1]}
    return dict(input_channels=ic, node_embedding_size=m["hidden"], message_passing_layers=m["layers"], dropout=0.0,
                heads=m["heads"], concat_path=m["concat_path"], bl_features=m["bl_features"],
                divided_features=m["divided_features"], global_feats=False, mlp_layers=list(m["mlp_layers"]),
                act="torch.nn.PReLU()", mlp_head_act=None, mlp_bn=False)


def _model(fx):
    from hgin import HetroGAT
    model = HetroGAT(**_kwargs(fx))
    model.load_state_dict({k[3:]: v for k, v in fx.items() if k.startswith("sd.")})   # materialises the lazy weights
    return model.to(DEV).train()


def _close(a, b, tol=1e-5):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return bool(((a - b).abs() <= tol + tol * b.abs()).all())


@pytest.mark.parametrize("case", CASES)
def test_attention_and_aggregate_vs_reference(case):
    """Per relation: the attention of every edge of the self-loop-adjusted edge list and the pre-bias aggregate."""
    from hgin import _lib
    from hgin.gat import _GatAttentionFn, _logits, gat_graph
    from hgin.ops import _p, _stream
    fx = load_fixture(case)
    model = _model(fx)
    x, ei, _, _ = fixture_inputs(fx, DEV)
    model._select_features(x)
    with torch.no_grad():
        for key, conv in model.convs[0].convs.items():
            src, _, dst = key.split("__")
            xs, xd = conv.lin_src(x[src]), conv.lin_dst(x[dst])
            H, C = conv.heads, conv.out_channels
            g = gat_graph(ei[(src, key.split("__")[1], dst)], xs.size(0), xd.size(0), True)
            with _lib.trace_launches() as tr:
                agg = _GatAttentionFn.apply(xs, xd, conv.att_src, conv.att_dst, None, None, g, H, C, 0.2)
            assert any(t.startswith("k_gat_attn_w<") for t in tr.kernels), tr.kernels  # the one-pass form
            want = fx[f"agg.0.{key}"]
            assert _close(agg.view(-1, H, C), want), (key, float((agg.cpu().view(-1, H, C) - want).abs().max()))
            # alpha of CSR position p belongs to edge perm[p] of the adjusted list
            alpha = torch.empty(g.n_edges, H, device=DEV)
            a_s = _logits(xs, conv.att_src.reshape(-1).contiguous(), H, C)
            a_d = _logits(xd, conv.att_dst.reshape(-1).contiguous(), H, C)
            out = torch.empty(xd.size(0), H * C, device=DEV)
            _lib.call("hgin_gat_fwd_f32", _p(g.csr.rowptr), _p(g.csr.col), xd.size(0), H, C, _p(xs), xs.stride(0),
                      _p(a_s), _p(a_d), ctypes.c_float(0.2), None, None, 0, _p(alpha), _p(out), out.stride(0),
                      _stream(xs))
            ref_alpha = fx[f"alpha.0.{key}"][g.csr.perm.long().cpu()]
            assert _close(alpha, ref_alpha), (key, float((alpha.cpu() - ref_alpha).abs().max()))
            # the one-pass kernel's alpha and output against the same fixture (a_s formed from the x_s rows)
            alpha1, out1 = torch.empty_like(alpha), torch.empty_like(out)
            _lib.call("hgin_gat_attn_fwd_f32", _p(g.csr.rowptr), _p(g.csr.col), xd.size(0), H, C, _p(xs),
                      xs.stride(0), _p(conv.att_src.reshape(-1).contiguous()), _p(a_d), ctypes.c_float(0.2), None,
                      None, 0, _p(alpha1), _p(out1), out1.stride(0), _stream(xs))
            assert _close(alpha1, ref_alpha), (key, float((alpha1.cpu() - ref_alpha).abs().max()))
            assert _close(out1.view(-1, H, C), want), key


@pytest.mark.parametrize("case", CASES)
def test_forward_backward_step_vs_reference(case):
    fx = load_fixture(case)
    model = _model(fx)
    x, ei, batch, y = fixture_inputs(fx, DEV)
    opt = torch.optim.Adam(lr=1e-3, params=model.parameters(), weight_decay=0)
    opt.zero_grad()
    out = model(x, ei, batch)
    assert _close(out, fx["out"]), float((out.detach().cpu() - fx["out"]).abs().max())
    lv = 100.0 * torch.mean(torch.abs((out - y.reshape(-1, 1)) / y.reshape(-1, 1)))
    assert _close(lv, fx["loss_value"])
    torch.sqrt(lv).backward()
    for n, p in model.named_parameters():
        want = fx[f"grad.{n}"]
        if want.numel() == 0:        # the reference left it None (its relation does not reach the readout)
            assert p.grad is None, n
            continue
        assert p.grad is not None, n
        d = (p.grad.detach().double().cpu() - want.double()).norm()
        assert float(d) <= 1e-4 * float(want.double().norm()) + 1e-7, (n, float(d), float(want.norm()))
    opt.step()
    for n, p in model.named_parameters():
        assert _close(p, fx[f"step.{n}"]), n


def test_lazy_projection_init_and_train_py_order():
    """train.py's order on the device: construct (lazy (-1, -1) projections uninitialised), .cuda(), Adam, then the
    first forward materialises lin_src / lin_dst per relation (glorot bounds) and a training step runs; the parameter
    names are the reference's."""
    from hgin import HetroGAT
    fx = load_fixture("gat_cfg1_h16")
    torch.manual_seed(1997)
    model = HetroGAT(**_kwargs(fx)).to(DEV).train()
    opt = torch.optim.Adam(lr=1e-3, params=model.parameters())
    assert [n for n, _ in model.named_parameters()] == fx["meta"]["param_names_before_forward"]
    x, ei, batch, y = fixture_inputs(fx, DEV)
    out = model(x, ei, batch)
    assert set(model.state_dict().keys()) == {k[3:] for k in fx if k.startswith("sd.")}
    for k, v in model.state_dict().items():
        assert tuple(v.shape) == tuple(fx["sd." + k].shape), k
    w = model.convs[0].convs["path__uses__link"].lin_src.weight
    bound = (6.0 / (w.size(0) + w.size(1))) ** 0.5
    assert float(w.abs().max()) <= bound and float(w.abs().max()) > 0.5 * bound
    loss = torch.sqrt(100.0 * torch.mean(torch.abs((out - y.reshape(-1, 1)) / y.reshape(-1, 1))))
    loss.backward()
    opt.step()
    assert torch.isfinite(out).all()


def test_later_layers_reject_multi_head_inputs_like_the_reference():
    """models.py:425 builds GATConv(H, H) for layers > 1, fed the first layer's H * heads columns: the reference's
    F.linear raises; so does the drop-in (and with heads = 1 two layers run)."""
    from hgin import HetroGAT
    fx = load_fixture("gat_cfg1_h16")
    x, ei, batch, _ = fixture_inputs(fx, DEV)
    kw = _kwargs(fx)
    kw["message_passing_layers"] = 2
    model = HetroGAT(**kw).to(DEV)
    with pytest.raises(RuntimeError, match="cannot be multiplied"):
        model(dict(x), ei, batch)
    kw["heads"] = 1
    model = HetroGAT(**kw).to(DEV)
    out = model(dict(x), ei, batch)
    assert out.shape == (x["path"].size(0), 1) and torch.isfinite(out).all()


@pytest.mark.parametrize("H,C", [(16, 8), (4, 16), (1, 8), (3, 6), (2, 2)])
def test_relation_forward_backward_vs_oracle(H, C):
    """One relation's attention forward + backward, both kernel forms (the wave-group form for C in {8, 16}; the
    thread-per-(row, head) form for C = 6, 2), against the oracle's GATConv restatement (oracle.pyg_cpu.gat_relation)
    evaluated in float64 with autograd: output within 1e-5 (abs + rel), every gradient within 1e-5 of its norm."""
    from hgin import _lib
    from hgin.gat import _GatAttentionFn, gat_graph
    from oracle.pyg_cpu import gat_relation
    gen = torch.Generator().manual_seed(100 * H + C)
    ns, nd, E = 700, 500, 6000
    ei = torch.stack([torch.randint(0, ns, (E,), generator=gen), torch.randint(0, nd, (E,), generator=gen)])
    ei[:, :40] = torch.arange(40).repeat(2, 1)                       # coincident indices: removed, then re-added
    xs, xd = torch.randn(ns, H * C, generator=gen), torch.randn(nd, H * C, generator=gen)
    att_s, att_d = 0.3 * torch.randn(1, H, C, generator=gen), 0.3 * torch.randn(1, H, C, generator=gen)
    bias, g_out = torch.randn(H * C, generator=gen), torch.randn(nd, H * C, generator=gen)
    ref = [t.double().requires_grad_() for t in (xs, xd, att_s, att_d, bias)]
    _, agg = gat_relation(ref[0].view(ns, H, C), ref[1].view(nd, H, C), ei, ref[2], ref[3])
    out_ref = agg.reshape(nd, H * C) + ref[4]
    out_ref.backward(g_out.double())
    dev = [t.to(DEV).requires_grad_() for t in (xs, xd, att_s, att_d, bias)]
    graph = gat_graph(ei.to(DEV), ns, nd, True)
    with _lib.trace_launches() as tr:
        out = _GatAttentionFn.apply(dev[0], dev[1], dev[2], dev[3], dev[4], None, graph, H, C, 0.2)
        out.backward(g_out.to(DEV))
        torch.cuda.synchronize()
    wave = C % 4 == 0   # the one-pass forward (k_gat_attn_w) + wave-group backward, else the thread forms
    for k in ("k_gat_logits", "k_gat_attn", "k_gat_bwd_dst", "k_gat_bwd_src"):
        assert any(t.startswith(k + "_w<") for t in tr.kernels) == wave, (k, tr.kernels)
    assert any(t == "k_gat_fwd" for t in tr.kernels) == (not wave), tr.kernels
    assert _close(out, out_ref), float((out.detach().cpu().double() - out_ref.detach()).abs().max())
    for name, a, b in zip(("x_s", "x_d", "att_src", "att_dst", "bias"), dev, ref):
        d = float((a.grad.double().cpu() - b.grad).norm())
        assert d <= 1e-5 * float(b.grad.norm()) + 1e-9, (name, d, float(b.grad.norm()))
