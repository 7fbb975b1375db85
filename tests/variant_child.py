"""Child process of tests/test_gpu_variants.py: one libhgin.so kernel variant (selected by the process-static
HGIN_* environment switch its parent set before this interpreter started) run on the reference fixtures.

Checks the fixture tolerances of tests/test_gpu_model.py (fp32 outputs within 1e-5, gradients within 1e-4 of
their norm) and saves the outputs and gradients so the parent can compare variants bit for bit.

    python tests/variant_child.py OUT.pt
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (HERE, ROOT, os.path.join(ROOT, "gnn-link-prediction_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402

from conftest import fixture_inputs, fixture_model_kwargs, fixture_state_dict, load_fixture  # noqa: E402
from hgin import HetroGIN  # noqa: E402
from hgin.train import mape  # noqa: E402


def run(case):
    fx = load_fixture(case)
    model = HetroGIN(**fixture_model_kwargs(fx))
    model.load_state_dict(fixture_state_dict(fx))
    model = model.to("cuda").train()
    x, ei, batch, y = fixture_inputs(fx, "cuda")
    out = model(dict(x), ei, batch)
    ref = fx["out"].double()
    d = (out.detach().double().cpu() - ref).abs()
    assert bool((d <= 1e-5 + 1e-5 * ref.abs()).all()), (case, float(d.max()))
    torch.sqrt(mape(out, y.reshape(-1, 1))).backward()
    no_grad = set(fx["meta"]["no_grad_params"])
    g_scale = max(float(fx["grad." + n].double().norm()) for n, _ in model.named_parameters() if n not in no_grad)
    res = {"out": out.detach().cpu()}
    for n, p in model.named_parameters():
        if n in no_grad:
            assert p.grad is None, n
            continue
        r = fx["grad." + n].double()
        err = float((p.grad.double().cpu() - r).norm())
        assert err <= 1e-4 * float(r.norm()) + 1e-6 * g_scale, (case, n, err)
        res["grad." + n] = p.grad.detach().cpu()
    return res


def main():
    torch.cuda.init()
    res = {case: run(case) for case in ("cfg1_L2", "w128_L2", "wide_L3", "w256_L3")}
    torch.save(res, sys.argv[1])
    print("variant ok", {k: v for k, v in os.environ.items() if k.startswith("HGIN_")}, flush=True)


if __name__ == "__main__":
    main()
