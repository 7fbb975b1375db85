"""Where does autograd add gradients in a HetroGIN step?  Profiles one backward of a small cfg3-schema model with
torch.profiler (record_shapes) and prints every aten::add / add_ with its input shapes and the autograd node
it runs under."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gnn-link-prediction_amd")]
import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

from hgin import HetroGIN  # noqa: E402
from hgin.data import CONFIGS, scaled_config, synthetic_graph  # noqa: E402

cfg = scaled_config(CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "cfg3"], 0.01, name="small")
g = synthetic_graph(cfg, seed=0, device="cuda")
torch.manual_seed(1997)
model = HetroGIN(**cfg.model_kwargs({"link": cfg.f_link, "path": cfg.f_path, "node": cfg.f_node})).cuda()
print({t: tuple(v.shape) for t, v in g.x.items()})
for it in range(2):
    model.zero_grad(set_to_none=True)
    _, lv = model.forward_loss(g.x_dict(), g.edge_index_dict(), g.batch["path"], g.y)
    loss = torch.sqrt(lv)
    if it == 0:
        loss.backward()
        continue
    with profile(activities=[ProfilerActivity.CPU], record_shapes=True, with_stack=False) as prof:
        loss.backward()
    names = {}
    for ev in prof.events():
        names[ev.name] = names.get(ev.name, 0) + 1
    print(sorted(names.items()))
    for ev in prof.events():
        if "add" in ev.name or ev.name in ("aten::sum", "aten::stack", "aten::copy_"):
            par = ev.cpu_parent
            chain = []
            while par is not None and len(chain) < 4:
                chain.append(par.name)
                par = par.cpu_parent
            print(ev.name, ev.input_shapes, " <- ", " <- ".join(chain))
