"""End-to-end parity of the HIP HetroGIN against the golden vectors produced by the reference's own
models.py, and against the CPU oracle over several optimizer steps.

Tolerances (BASELINE.json north star): index / CSR work and the aggregates bit-exact; fp32 embeddings and
outputs within 1e-5 (abs + rel); gradients (which pass through fp32 GEMMs of different summation order)
within 1e-4 relative of their norm."""
import re

import pytest
import torch

from conftest import CASES, fixture_inputs, fixture_model_kwargs, fixture_state_dict, is_compact, load_fixture
from hgin import HetroGIN, _lib, ops
from hgin.train import mape
from oracle.pyg_cpu import OracleHetroGIN, train_step

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _close(a, b, tol=1e-5):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return bool(((a - b).abs() <= tol + tol * b.abs()).all())


def _rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).norm() / (b.norm() + 1e-30))


def _model_from_fixture(fx):
    model = HetroGIN(**fixture_model_kwargs(fx))
    model.load_state_dict(fixture_state_dict(fx))
    return model.to(DEV).train()


def _sums(t):
    d = t.detach().double().cpu()
    return torch.stack([d.sum(), d.abs().sum(), (d * d).sum()])


def _close_sums(got, want, tol):
    """Whole-tensor float64 (sum, sum|v|, sum v^2) of a compact fixture: the plain sum within tol of sum|v|."""
    return (abs(float(got[0] - want[0])) <= tol * float(want[1]) and
            abs(float(got[1] - want[1])) <= tol * float(want[1]) and
            abs(float(got[2] - want[2])) <= 2 * tol * float(want[2]))


def _layer_input(fx, li, key, n_src):
    """Layer li >= 1 input of a compact fixture's relation: the reference's layer li-1 output at every source
    row the sampled aggregate rows read, zeros elsewhere (those rows feed no sampled destination)."""
    x = torch.zeros(n_src, fx[f"src.{li}.{key}"].shape[1])
    x[fx[f"rows.src.{li}.{key}"]] = fx[f"src.{li}.{key}"]
    return x.to(DEV)


# the kernels the headline width runs (K = 512 first layer, K = N = 256 above it), as trace tags
W256_KERNELS = (r"k_gemm_nt<EPI1,\d+x\d+,split,N256,K512>",                # first layer forward (eps-scaled self half)
                r"k_wss_f32<EPI1,[01],[01]>",                               # layers 1-2 forward (staggered)
                r"k_wsp_f32<256,256,prelu_bwd_fused>",                      # dW + PReLU bwd (g_z out): every layer
                r"k_wsp_f32<256,256>",                                      # first layer dW, columns [256, 512)
                r"k_wss_f32<EPI4,1,[01]>")                                  # layers 1-2 dX + self-term backward


@pytest.mark.parametrize("case", CASES)
def test_aggregates_bit_exact_every_layer(case):
    """Every propagate() result of the reference, recomputed by the HIP aggregate from the same layer input."""
    fx = load_fixture(case)
    model = _model_from_fixture(fx)
    x, ei, batch, _ = fixture_inputs(fx, DEV)
    captured = {}

    def grab(module, args):
        captured["x0"] = dict(args[0])

    h = model.convs[0].register_forward_pre_hook(grab)
    with torch.no_grad():
        model(dict(x), ei, batch)
    h.remove()
    compact = is_compact(fx)
    sizes = {t: v.size(0) for t, v in x.items()}
    for li, conv in enumerate(model.convs):
        if li == 0:
            xin = captured["x0"]
        elif not compact:
            xin = {t: fx[f"layer.{li - 1}.{t}"].to(DEV) for t in ("path", "link", "node")}
        for key in conv.convs.keys():
            src, rel, dst = key.split("__")
            xs = _layer_input(fx, li, key, sizes[src]) if (compact and li > 0) else xin[src]
            graph = ops.relation_graph(ei[(src, rel, dst)], sizes[src], sizes[dst])
            agg = ops.aggregate(xs, None, None, graph, ops.COMBINE_NONE).cpu()
            k = f"agg.{li}.{key}"
            if compact:      # sampled rows (incl. the max- and a zero-in-degree one) bit-exact
                assert torch.equal(agg[fx["rows." + k]], fx[k]), (li, key)
                if li == 0:
                    assert _close_sums(_sums(agg), fx["sums." + k], 1e-12), (li, key)
            else:
                assert torch.equal(agg, fx[k]), (li, key)


@pytest.mark.parametrize("case", CASES)
def test_forward_backward_step_vs_reference(case):
    fx = load_fixture(case)
    model = _model_from_fixture(fx)
    x, ei, batch, y = fixture_inputs(fx, DEV)
    outs = {}
    hooks = [c.register_forward_hook(lambda m, i, o, li=li: outs.__setitem__(li, o)) for li, c in
             enumerate(model.convs)]
    opt = torch.optim.Adam(lr=1e-3, params=model.parameters(), weight_decay=0)
    opt.zero_grad()
    compact = is_compact(fx)
    with _lib.trace_launches() as tr:
        out = model(dict(x), ei, batch)
        for h in hooks:
            h.remove()
        lv = mape(out, y.reshape(-1, 1))
        torch.sqrt(lv).backward()
    torch.cuda.synchronize()
    for li, o in outs.items():
        for t, v in o.items():
            k = f"layer.{li}.{t}"
            if compact:
                # Headline width (K = 512, 3 layers): the fp32 reference itself is more than 1e-5 (abs + rel) from
                # exact arithmetic on a few layer-2 elements (tests/golden/w256_L3.pt meta
                # "reference_fp32_vs_exact": 64 of 20M), so no fp32 evaluation can be elementwise within 1e-5 of
                # it everywhere.  Bound: every sampled element within 1e-5 (abs + rel) of the float64 reference
                # plus the fp32 reference's own deviation there (the sampled rows include its 8 worst); the rows
                # within 1e-5 relative L2 of the fp32 reference; whole-tensor sums within 1e-5 of sum |v|.
                got = v[fx["rows." + k].to(DEV)].detach().double().cpu()
                e, r = fx["exact." + k], fx[k].double()
                assert ((got - e).abs() <= 1e-5 * (1 + e.abs()) + (r - e).abs()).all(), (li, t)
                assert float((got - r).norm() / r.norm()) <= 1e-5, (li, t)
                assert _close_sums(_sums(v), fx["sums." + k], 1e-5), (li, t)
                print(f"[w256] layer {li} {t}: max |hip - fp32 ref| {float((got - r).abs().max()):.3g}, "
                      f"max |hip - exact| {float((got - e).abs().max()):.3g}, "
                      f"max |fp32 ref - exact| {float((r - e).abs().max()):.3g}")
            else:
                assert _close(v, fx[k]), (li, t)          # fp32 embeddings within 1e-5
    assert _close(out, fx["out"])
    assert _close(lv, fx["loss_value"])
    if compact:
        print(f"[w256] out: max |hip - fp32 ref| {float((out.detach().cpu() - fx['out']).abs().max()):.3g}, "
              f"max |hip - exact| {float((out.detach().cpu().double() - fx['exact.out']).abs().max()):.3g}")
    if case == "w256_L3":   # the headline's kernels ran inside this parity check
        missing = [k for k in W256_KERNELS if not any(re.fullmatch(k, t) for t in tr.kernels)]
        assert not missing, (missing, sorted(set(tr.kernels)))
        # no separate PReLU-backward pass at the GIN width (the fp32 step folds it into every dW GEMM)
        assert "k_rows_bwd<0,f32,N256>" not in tr.kernels, sorted(set(tr.kernels))
    no_grad = set(fx["meta"]["no_grad_params"])
    g_scale = max(float(fx["grad." + n].double().norm()) for n, _ in model.named_parameters() if n not in no_grad)
    grads = {}
    for n, p in model.named_parameters():
        if n in no_grad:
            assert p.grad is None, n                                   # dead relations: no gradient, as in PyG
            continue
        ref = fx["grad." + n]
        grads[n] = ref
        # 1e-4 of the gradient's norm, with a floor of 1e-6 of the model's largest gradient norm for gradients
        # that are identically zero in exact arithmetic (a Linear bias feeding a training-mode BatchNorm: both
        # sides are rounding noise)
        err = float((p.grad.double().cpu() - ref.double()).norm())
        assert err <= 1e-4 * float(ref.double().norm()) + 1e-6 * g_scale, (n, err, float(ref.norm()))
    if compact:
        return                 # compact fixtures carry no Adam step
    opt.step()
    for n, p in model.named_parameters():
        ref = fx["step." + n]
        if n in no_grad:
            assert torch.equal(p.detach().cpu(), ref), n
            continue
        g = grads[n].abs().double()
        # Adam's first step moves each weight by ~lr * sign(g): where |g| is within the gradient error bound
        # asserted above, the sign may legitimately differ and the weight may move by up to 2 * lr.
        bound = 1e-4 * float(g.norm()) + 1e-6 * g_scale
        tol = torch.where(g > bound, torch.full_like(g, 2e-5), torch.full_like(g, 2.1e-3)).float()
        assert ((p.detach().cpu() - ref).abs() <= tol).all(), n


def test_training_trajectory_vs_oracle():
    """Five train.py steps on cfg1 (GPU) track the CPU oracle's loss trajectory."""
    fx = load_fixture("cfg1_L2")
    x, ei, batch, y = fixture_inputs(fx)
    torch.manual_seed(1997)
    ref = OracleHetroGIN(**fixture_model_kwargs(fx))
    ref_opt = torch.optim.Adam(lr=1e-3, params=ref.parameters())
    model = _model_from_fixture(fx)
    opt = torch.optim.Adam(lr=1e-3, params=model.parameters())
    xg, eig, bg, yg = fixture_inputs(fx, DEV)
    for step in range(5):
        l_ref = float(train_step(ref, ref_opt, dict(x), ei, batch, y))
        opt.zero_grad()
        out = model(dict(xg), eig, bg)
        lv = mape(out, yg.reshape(-1, 1))
        torch.sqrt(lv).backward()
        opt.step()
        assert abs(float(lv) - l_ref) <= 1e-4 * abs(l_ref), (step, float(lv), l_ref)


def test_deterministic_runs():
    fx = load_fixture("w128_L2")
    res = []
    for _ in range(2):
        model = _model_from_fixture(fx)
        x, ei, batch, y = fixture_inputs(fx, DEV)
        out = model(dict(x), ei, batch)
        torch.sqrt(mape(out, y.reshape(-1, 1))).backward()
        res.append([out.detach().clone()] + [p.grad.clone() for p in model.parameters() if p.grad is not None])
    for a, b in zip(*res):
        assert torch.equal(a, b)


def test_prune_dead_same_output_and_grads():
    fx = load_fixture("wide_L3")
    x, ei, batch, y = fixture_inputs(fx, DEV)
    full = _model_from_fixture(fx)
    pruned = _model_from_fixture(fx)
    pruned.prune_dead(True)
    o1, o2 = full(dict(x), ei, batch), pruned(dict(x), ei, batch)
    assert torch.equal(o1, o2)
    torch.sqrt(mape(o1, y.reshape(-1, 1))).backward()
    torch.sqrt(mape(o2, y.reshape(-1, 1))).backward()
    for (n, p1), (_, p2) in zip(full.named_parameters(), pruned.named_parameters()):
        assert (p1.grad is None) == (p2.grad is None), n
        if p1.grad is not None:
            assert torch.equal(p1.grad, p2.grad), n


def test_full_size_cfg2_step():
    """One full cfg2 (1M nodes / 10M edges, H=128, L=2) training step: finite loss, size-independent checks."""
    from hgin.data import CONFIGS, synthetic_graph
    from hgin.train import train_step as hip_step
    cfg = CONFIGS["cfg2"]
    g = synthetic_graph(cfg, seed=0, device=DEV)
    torch.manual_seed(1997)
    model = HetroGIN(**cfg.model_kwargs({"link": cfg.f_link, "path": cfg.f_path, "node": cfg.f_node})).to(DEV)
    opt = torch.optim.Adam(lr=1e-3, params=model.parameters())
    l0 = float(hip_step(model, opt, g))
    l1 = float(hip_step(model, opt, g))
    assert torch.isfinite(torch.tensor([l0, l1])).all()
    # aggregate of all-ones features = in-degree (exact small integers), the largest relation
    e = g.edge_index[("path", "uses", "link")]
    graph = ops.relation_graph(e, cfg.n_path, cfg.n_link)
    ones = torch.ones(cfg.n_path, 128, device=DEV)
    agg = ops.aggregate(ones, None, None, graph, ops.COMBINE_NONE)
    deg = torch.bincount(e[1], minlength=cfg.n_link).float()
    assert torch.equal(agg, deg[:, None].expand(-1, 128))
    # against torch's own device scatter (atomics, so a tolerance)
    x = g.x["path"]
    ref = torch.zeros(cfg.n_link, 128, device=DEV).index_add_(0, e[1], x[e[0]])
    agg = ops.aggregate(x, None, None, graph, ops.COMBINE_NONE)
    assert torch.allclose(agg, ref, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("feat", ["f32", "bf16"])
def test_captured_static_step_equals_eager(feat):
    """bench.py's default mode: a hipGraph replay of the whole step (forward, fused head + loss, backward,
    capturable Adam) runs the eager step's kernels in the same order -> bitwise the same trajectory."""
    import dataclasses

    from hgin.data import CONFIGS, scaled_config, synthetic_graph
    from hgin.graphs import CapturedStaticStep
    from hgin.train import train_step as hip_step
    cfg = dataclasses.replace(scaled_config(CONFIGS["cfg2"], 0.02, name="cfg2-small"), feat_dtype=feat)
    g = synthetic_graph(cfg, seed=0, device=DEV)
    runs = []
    for mode in ("eager", "graph"):
        torch.manual_seed(1997)
        model = HetroGIN(**cfg.model_kwargs({"link": cfg.f_link, "path": cfg.f_path, "node": cfg.f_node})).to(DEV)
        opt = torch.optim.Adam(lr=1e-3, params=model.parameters(), capturable=True)
        if mode == "eager":
            losses = [hip_step(model, opt, g).clone() for _ in range(3)]
        else:
            st = CapturedStaticStep(model, opt, g, warmup=1)
            losses = [torch.zeros(())] + [st.step().clone() for _ in range(2)]
        torch.cuda.synchronize()
        runs.append((losses, [p.detach().clone() for p in model.parameters()]))
    (l_e, p_e), (l_g, p_g) = runs
    assert torch.equal(l_e[2], l_g[2]) and torch.equal(l_e[1], l_g[1])
    for a, b in zip(p_e, p_g):
        assert torch.equal(a, b)


@pytest.mark.parametrize("case", ["cfg1_L2", "collate2_global_bn"])
def test_evaluate_host_resident_call(case):
    """train.py:322-348 unchanged: load_model on the CPU -> load_state_dict -> eval -> model(cpu batch) under
    set_grad_enabled(False).  The call runs on the MI355X and returns the output on the CPU, within 1e-5 of
    the reference's (eval-mode BatchNorm: against the oracle's eval-mode output); the parameters stay on the
    host; a host-resident call that records gradients raises (training moves the model first)."""
    fx = load_fixture(case)
    kw = fixture_model_kwargs(fx)
    model = HetroGIN(**kw)
    sd = fixture_state_dict(fx)
    model.load_state_dict(sd)
    model.eval()
    x, ei, batch, y = fixture_inputs(fx)
    with torch.set_grad_enabled(False):
        out = model(dict(x), ei, batch)
        out2 = model(dict(x), ei, batch)
    assert out.device.type == "cpu" and torch.equal(out, out2)    # bitwise run to run (global pooling included)
    assert all(p.device.type == "cpu" for p in model.parameters())
    assert all(b.device.type == "cpu" for b in model.buffers())
    if fx["meta"]["mlp_bn"]:
        ref = OracleHetroGIN(**fixture_model_kwargs(fx))
        ref.load_state_dict(sd)
        ref.eval()
        with torch.no_grad():
            want = ref(dict(x), ei, batch)
    else:
        want = fx["out"]
    assert _close(out, want)
    # the device copies of the weights persist between calls and follow every change of the host weights:
    # load_state_dict (in place) and an in-place edit of one parameter
    from hgin.models import _LENT
    dev_copies = {k: v[1].data_ptr() for k, v in _LENT[model].items()}
    with torch.set_grad_enabled(False):
        model(dict(x), ei, batch)
    assert {k: v[1].data_ptr() for k, v in _LENT[model].items()} == dev_copies   # no re-copy
    sd2 = {k: (v * 1.01 if v.is_floating_point() else v) for k, v in sd.items()}
    model.load_state_dict(sd2)
    with torch.no_grad():
        next(model.parameters()).mul_(0.5)
        out3 = model(dict(x), ei, batch)
        fresh = HetroGIN(**fixture_model_kwargs(fx))
        fresh.load_state_dict(model.state_dict())
        fresh.eval()
        out4 = fresh(dict(x), ei, batch)
    assert torch.equal(out3, out4) and not torch.equal(out3, out)
    # an edit through .data does not bump the parameter's version counter: still followed
    next(model.parameters()).data.mul_(2.0)
    with torch.no_grad():
        out5 = model(dict(x), ei, batch)
        fresh.load_state_dict(model.state_dict())
        out6 = fresh(dict(x), ei, batch)
    assert torch.equal(out5, out6) and not torch.equal(out5, out3)
    from hgin.models import release_device_cache
    release_device_cache(model)
    assert model not in _LENT
    model.train()
    with pytest.raises(RuntimeError, match="gradients enabled"):
        model(dict(x), ei, batch)


@pytest.mark.parametrize("feat", ["f32", "bf16"])
def test_layer_fn_equals_per_relation_autograd(feat):
    """The one-node-per-layer backward (conv.LAYER_FN, ops._HeteroGINLayerFn: shared-node-type gradient sums
    inside the CSC aggregate / dX epilogue) against one autograd node per relation (autograd adds them):
    the same contributions summed in another order (autograd's input-buffer order is not the relations' reverse
    order everywhere): fp32 within 1e-6 relative L2; bf16 within 1e-2 (the fused sum also rounds once instead of
    twice, and later bf16 GEMMs amplify the one-ulp differences)."""
    import dataclasses

    from hgin import conv as conv_mod
    from hgin.data import CONFIGS, scaled_config, synthetic_graph
    cfg = dataclasses.replace(scaled_config(CONFIGS["cfg3"], 0.003, name="cfg3-small"), feat_dtype=feat)
    g = synthetic_graph(cfg, seed=0, device=DEV)
    res = []
    for on in (True, False):
        conv_mod.LAYER_FN = on
        try:
            torch.manual_seed(1997)
            model = HetroGIN(**cfg.model_kwargs({"link": cfg.f_link, "path": cfg.f_path, "node": cfg.f_node})).to(DEV)
            # gradient-carrying inputs, so every layer's input gradients (the summed ones) are exercised
            x = {t: v.clone().requires_grad_(True) for t, v in g.x.items()}
            _, lv = model.forward_loss(dict(x), g.edge_index_dict(), g.batch["path"], g.y)
            torch.sqrt(lv).backward()
            res.append([lv.detach()] + [x[t].grad for t in ("path", "link", "node")] +
                       [p.grad for p in model.parameters()])
        finally:
            conv_mod.LAYER_FN = True
    for a, b in zip(*res):
        assert (a is None) == (b is None)
        if a is None:
            continue
        rel = float((a.double() - b.double()).norm() / (b.double().norm() + 1e-30))
        assert rel <= (1e-6 if feat == "f32" else 1e-2), rel


def test_lazy_self_term_gradient_is_bitwise_the_materialised_one():
    """ops._LazySelf (the first ADD-mode dX of a node type writes no g_x_dst; the next CSC aggregate of that type
    applies fl(1 + eps) C as its own self term) against the materialised g_x_dst: every input and parameter
    gradient bitwise equal at the headline width (fp32, K = N = 256 above the first layer), and the lazy run's
    dX GEMMs without the g_x_dst stream (k_wss_f32<EPI4,1,0>) outnumber the materialised run's."""
    import dataclasses
    import re

    from hgin.data import CONFIGS, scaled_config, synthetic_graph
    cfg = dataclasses.replace(scaled_config(CONFIGS["cfg3"], 0.003, name="cfg3-small"), feat_dtype="f32")
    g = synthetic_graph(cfg, seed=0, device=DEV)
    res, n_nogd = [], []
    for on in (True, False):
        ops.LAZY_SELF = on
        try:
            torch.manual_seed(1997)
            model = HetroGIN(**cfg.model_kwargs({"link": cfg.f_link, "path": cfg.f_path, "node": cfg.f_node})).to(DEV)
            x = {t: v.clone().requires_grad_(True) for t, v in g.x.items()}
            with _lib.trace_launches() as tr:
                _, lv = model.forward_loss(dict(x), g.edge_index_dict(), g.batch["path"], g.y)
                torch.sqrt(lv).backward()
            torch.cuda.synchronize()
            n_nogd.append(sum(1 for t in tr.kernels if re.match(r"k_wss_f32<EPI4,1,0>", t)))
            res.append([lv.detach()] + [x[t].grad for t in ("path", "link", "node")] +
                       [p.grad for p in model.parameters()])
        finally:
            ops.LAZY_SELF = True
    assert n_nogd[0] > n_nogd[1], n_nogd
    for a, b in zip(*res):
        assert (a is None) == (b is None)
        if a is not None:
            assert torch.equal(a, b)


def test_global_feats_bitwise_deterministic_and_no_aten_scatter():
    """GLOBAL_FEATS (models.py:347-352) on the collated two-graph fixture: the pooling runs on hgin_global_pool_f32
    (launch trace), the forward output and every gradient are bitwise identical run to run."""
    fx = load_fixture("collate2_global_bn")
    res = []
    for _ in range(2):
        model = _model_from_fixture(fx)
        x, ei, batch, y = fixture_inputs(fx, DEV)
        with _lib.trace_launches() as tr:
            out = model(dict(x), ei, batch)
            torch.sqrt(mape(out, y.reshape(-1, 1))).backward()
        torch.cuda.synchronize()
        assert any(t.startswith("k_seg_pool<f32") for t in tr.kernels), tr.kernels
        res.append([out.detach().clone()] + [p.grad.clone() for p in model.parameters() if p.grad is not None])
    for a, b in zip(*res):
        assert torch.equal(a, b)
