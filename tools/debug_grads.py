"""Diagnostic: per-parameter gradient error of the HIP HetroGIN vs the oracle (float64 CPU) on a fixture."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gnn-link-prediction_amd"), os.path.join(ROOT, "tests")]

import torch  # noqa: E402

from conftest import fixture_inputs, fixture_model_kwargs, load_fixture  # noqa: E402
from hgin import HetroGIN  # noqa: E402
from hgin.train import mape  # noqa: E402
from oracle.pyg_cpu import OracleHetroGIN  # noqa: E402

case = sys.argv[1] if len(sys.argv) > 1 else "cfg1_L2"
fx = load_fixture(case)
sd = {k[3:]: v for k, v in fx.items() if k.startswith("sd.")}
ref = OracleHetroGIN(**fixture_model_kwargs(fx)).double()
ref.load_state_dict(sd)
x, ei, batch, y = fixture_inputs(fx)
out_r = ref({k: v.double() for k, v in x.items()}, ei, batch)
torch.sqrt(mape(out_r, y.double().reshape(-1, 1))).backward()

m = HetroGIN(**fixture_model_kwargs(fx))
m.load_state_dict(sd)
m = m.cuda()
xg, eig, bg, yg = fixture_inputs(fx, "cuda")
out = m(dict(xg), eig, bg)
torch.sqrt(mape(out, yg.reshape(-1, 1))).backward()
print("out rel", float((out.double().cpu() - out_r).norm() / out_r.norm()))
for (n, p), (_, q) in zip(m.named_parameters(), ref.named_parameters()):
    if q.grad is None:
        print(f"{n:60s} ref None, hip {'None' if p.grad is None else 'SET'}")
        continue
    r = float((p.grad.double().cpu() - q.grad).norm() / (q.grad.norm() + 1e-300))
    print(f"{n:60s} rel {r:.3e}  |g| {float(q.grad.norm()):.3e}")
