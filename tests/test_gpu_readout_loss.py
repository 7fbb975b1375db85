"""§8 F3 on the GPU: the fused readout head + MAPE loss (hgin_head_mape_*) against the reference expression
(train.py:12-13 mape over models.py's head Linear) evaluated in float64 on the same inputs, and the fused
training step against the reference fixtures."""
import numpy as np
import pytest
import torch

from conftest import fixture_inputs, fixture_model_kwargs, fixture_state_dict, load_fixture
from hgin import HetroGIN, ops
from hgin.train import mape, train_step

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _ref(h, w, b, y):
    hr = h.detach().double().requires_grad_()
    wr = w.detach().double().requires_grad_()
    br = b.detach().double().requires_grad_()
    out = hr @ wr.t() + br
    lv = 100.0 * torch.mean(torch.abs((out - y.double().reshape(-1, 1)) / y.double().reshape(-1, 1)))
    torch.sqrt(lv).backward()
    return out.detach(), lv.detach(), hr.grad, wr.grad, br.grad


@pytest.mark.parametrize("M,K,dtype", [(1, 1, torch.float32), (1000, 32, torch.float32), (600_001, 32, torch.float32),
                                       (777, 70, torch.float32), (5000, 32, torch.bfloat16),
                                       (300_000, 32, torch.bfloat16)])
def test_head_mape_vs_float64(M, K, dtype):
    g = torch.Generator(device=DEV).manual_seed(M + K)
    h = torch.randn(M, K, device=DEV, generator=g).to(dtype).requires_grad_()
    lin = torch.nn.Linear(K, 1).to(DEV)
    y = torch.rand(M, device=DEV, generator=g) + 0.5
    out, lv = ops.head_mape(h, lin.weight, lin.bias, y)
    assert out.shape == (M, 1) and out.dtype == torch.float32 and not out.requires_grad
    torch.sqrt(lv).backward()
    r_out, r_lv, r_gh, r_gw, r_gb = _ref(h, lin.weight, lin.bias, y)
    assert float((out.double() - r_out).abs().max()) <= 1e-5 * (float(r_out.abs().max()) + 1)
    assert abs(float(lv) - float(r_lv)) <= 1e-5 * float(r_lv)
    tol = 1e-5 if dtype == torch.float32 else 8e-3      # bf16 g_h is stored rounded (2^-8 relative)
    assert float((h.grad.double() - r_gh).norm()) <= tol * float(r_gh.norm()) + 1e-12
    assert float((lin.weight.grad.double() - r_gw).norm()) <= 1e-5 * float(r_gw.norm()) + 1e-9
    assert abs(float(lin.bias.grad) - float(r_gb)) <= 1e-5 * (float(r_gb.abs()) + 1e-6)


def test_head_mape_deterministic_and_no_sync_needed():
    h = torch.randn(200_000, 32, device=DEV, requires_grad=True)
    lin = torch.nn.Linear(32, 1).to(DEV)
    y = torch.rand(200_000, device=DEV) + 0.5
    res = []
    for _ in range(2):
        h.grad = None
        lin.zero_grad()
        out, lv = ops.head_mape(h, lin.weight, lin.bias, y)
        assert lv.device.type == "cuda"          # loss stays on the device (no .item())
        torch.sqrt(lv).backward()
        res.append((lv.clone(), h.grad.clone(), lin.weight.grad.clone(), lin.bias.grad.clone()))
    for a, b in zip(*res):
        assert torch.equal(a, b)


@pytest.mark.parametrize("case", ["cfg1_L2", "wide_L3", "w128_L2", "w256_L3"])
def test_fused_loss_matches_reference_fixture(case):
    fx = load_fixture(case)
    model = HetroGIN(**fixture_model_kwargs(fx))
    model.load_state_dict(fixture_state_dict(fx))
    model = model.to(DEV).train()
    x, ei, batch, y = fixture_inputs(fx, DEV)
    out, lv = model.forward_loss(dict(x), ei, batch, y)
    assert float((out.cpu().double() - fx["out"].double()).norm() / fx["out"].double().norm()) <= 1e-5
    assert abs(float(lv) - float(fx["loss_value"])) <= 1e-5 * abs(float(fx["loss_value"]))
    torch.sqrt(lv).backward()
    no_grad = set(fx["meta"]["no_grad_params"])
    g_scale = max(float(fx["grad." + n].double().norm()) for n, _ in model.named_parameters() if n not in no_grad)
    for n, p in model.named_parameters():
        if n in no_grad:
            assert p.grad is None, n
            continue
        ref = fx["grad." + n].double()
        err = float((p.grad.cpu().double() - ref).norm())
        assert err <= 1e-4 * float(ref.norm()) + 1e-6 * g_scale, (n, err, float(ref.norm()))


def test_fused_and_unfused_train_steps_agree():
    """train_step(fused_loss=True) vs the unfused train.py expression: same loss, same gradients."""
    from hgin.data import CONFIGS, scaled_config, synthetic_graph
    cfg = scaled_config(CONFIGS["cfg2"], 0.01)
    g = synthetic_graph(cfg, seed=3, device=DEV)
    res = []
    for fused in (True, False):
        torch.manual_seed(1997)
        m = HetroGIN(**cfg.model_kwargs({"link": 128, "path": 128, "node": 128})).to(DEV)
        opt = torch.optim.SGD(m.parameters(), lr=0.0)       # keep the parameters: compare gradients
        lv = float(train_step(m, opt, g, fused_loss=fused))
        res.append((lv, {n: p.grad.clone() for n, p in m.named_parameters() if p.grad is not None}))
    (l1, g1), (l2, g2) = res
    assert abs(l1 - l2) <= 1e-5 * abs(l2)
    assert g1.keys() == g2.keys()
    scale = max(float(v.norm()) for v in g2.values())
    for n in g1:
        assert float((g1[n] - g2[n]).norm()) <= 1e-4 * float(g2[n].norm()) + 1e-6 * scale, n
