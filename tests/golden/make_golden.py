"""Generate the golden fixtures under tests/golden/ by EXECUTING the reference's own ``models.py``.

Run in the build container only (the GPU box has no /root/reference):

    python tests/golden/make_golden.py            # writes tests/golden/<case>.pt

The reference's ``models.py`` imports PyG / torch_scatter / torch_sparse, which are absent from this
image.  ``tests/golden/pyg_shim`` restates the handful of PyG 2.0.2 symbols it touches
(see its README); everything HetroGIN itself owns (GINConv combine + concat, eps / PReLU init, the double
Linear initialisation through ``reset``, channel bookkeeping, feature slicing, readout, state_dict
layout) runs from the reference file.  ``sys.dont_write_bytecode`` keeps ``/root/reference`` untouched.

Each fixture is a flat dict of tensors (+ a ``meta`` dict of plain values), loadable with
``torch.load(path, weights_only=True)``:

* ``in.x.<type>``, ``in.ei.<src__rel__dst>``, ``in.batch``, ``in.y``   — inputs (relation order kept)
* ``sd.<key>``                 — the model's state_dict right after construction under seed 1997
* ``agg.<layer>.<relkey>``     — every propagate() result (pre-combine aggregate), per layer / relation
* ``layer.<layer>.<type>``     — HeteroConv outputs per layer and node type
* ``out``, ``loss_value``      — forward output [N_path, 1] and MAPE (train.py:12-13, :40)
* ``grad.<param>``             — .grad of every parameter after sqrt(MAPE).backward() (train.py:42-43)
* ``step.<param>``             — parameters after one Adam(lr=1e-3, wd=0) step (train.py:141-142, :44)
"""
from __future__ import annotations

import importlib.util
import os
import sys

sys.dont_write_bytecode = True

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REFERENCE_MODELS = "/root/reference/models.py"

sys.path.insert(0, os.path.join(HERE, "pyg_shim"))
sys.path.insert(0, os.path.join(REPO, "gnn-link-prediction_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402

from hgin.data import CONFIGS, GraphConfig, HeteroGraph, scaled_config, synthetic_graph  # noqa: E402
from oracle import collate_np  # noqa: E402


def collate(graphs):
    """PyG Batch.from_data_list, as restated independently in oracle/collate_np.py."""
    c = collate_np.collate([collate_np.from_graph(g) for g in graphs])
    return HeteroGraph({t: torch.from_numpy(v) for t, v in c["x"].items()},
                       {r: torch.from_numpy(e) for r, e in c["edge_index"].items()}, torch.from_numpy(c["y"]),
                       {t: torch.from_numpy(b) for t, b in c["batch"].items()})


def load_reference_models():
    spec = importlib.util.spec_from_file_location("reference_models", REFERENCE_MODELS)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def run_case(ref, name: str, cfg: GraphConfig, graph, seed_model: int = 1997, mlp_bn: bool = False,
             global_feats: bool = False):
    torch.manual_seed(seed_model)
    input_channels = {"link": graph.x["link"].shape[1], "path": graph.x["path"].shape[1],
                      "node": graph.x["node"].shape[1]}
    kw = cfg.model_kwargs(input_channels)
    kw["mlp_bn"] = mlp_bn
    kw["global_feats"] = global_feats
    model = ref.HetroGIN(**kw)
    model.train()
    fx = {"meta": {"case": name, "config": cfg.name, "hidden": cfg.hidden, "layers": cfg.layers,
                   "divided_features": cfg.divided_features, "bl_features": cfg.bl_features,
                   "concat_path": cfg.concat_path, "global_feats": global_feats, "mlp_bn": mlp_bn,
                   "mlp_layers": list(cfg.mlp_layers), "seed_model": seed_model,
                   "input_channels_after_ctor": dict(input_channels),
                   "generator": "hgin.data.synthetic_graph (SURVEY.md §8.D)",
                   "reference": "models.py executed via tests/golden/pyg_shim"}}
    for t, v in graph.x.items():
        fx[f"in.x.{t}"] = v.clone()
    for et, e in graph.edge_index.items():
        fx[f"in.ei.{'__'.join(et)}"] = e.clone()
    fx["in.y"] = graph.y.clone()
    fx["in.batch"] = graph.batch["path"].clone()
    fx["meta"]["relations"] = ["__".join(et) for et in graph.edge_index.keys()]
    for k, v in model.state_dict().items():
        fx[f"sd.{k}"] = v.clone()

    layer_outs = []
    hooks = [conv.register_forward_hook(lambda m, i, o, li=li: layer_outs.append((li, o)))
             for li, conv in enumerate(model.convs)]
    opt = torch.optim.Adam(lr=1e-3, params=model.parameters(), weight_decay=0)
    opt.zero_grad()
    out = model(graph.x_dict(), graph.edge_index_dict(), graph.batch["path"])
    label = graph.y.reshape(-1, 1)
    loss_value = 100.0 * torch.mean(torch.abs((out - label) / label))  # train.py:12-13
    loss = torch.sqrt(loss_value)
    loss.backward()
    for h in hooks:
        h.remove()
    for li, conv in enumerate(model.convs):
        for key, layer in conv.convs.items():
            tr = layer.conv.trace
            assert len(tr) == 1, (key, len(tr))
            fx[f"agg.{li}.{key}"] = tr[0]
    for li, o in layer_outs:
        for t, v in o.items():
            fx[f"layer.{li}.{t}"] = v.detach().clone()
    fx["out"] = out.detach().clone()
    fx["loss_value"] = loss_value.detach().clone()
    for n, p in model.named_parameters():
        fx[f"grad.{n}"] = (p.grad.clone() if p.grad is not None else torch.zeros(0))
        fx["meta"].setdefault("no_grad_params", [])
        if p.grad is None:
            fx["meta"]["no_grad_params"].append(n)
    opt.step()
    for n, p in model.named_parameters():
        fx[f"step.{n}"] = p.detach().clone()
    torch.save(fx, os.path.join(HERE, f"{name}.pt"))
    return fx


def main():
    ref = load_reference_models()
    torch.set_num_threads(1)
    cfg1 = CONFIGS["cfg1"]
    # configs[0]: SURVEY cfg1 (H=8, L=2, config.json flags)
    run_case(ref, "cfg1_L2", cfg1, synthetic_graph(cfg1, seed=0))
    # config.json exactly (MP_LAYERS=1)
    import dataclasses
    run_case(ref, "cfg1_L1", dataclasses.replace(cfg1, layers=1), synthetic_graph(cfg1, seed=1))
    # divided + bl features, wide F, 3 layers (add-mode layers), with the unconvolved p->n and n->p
    wide = dataclasses.replace(scaled_config(CONFIGS["cfg2"], 1e-3, name="cfg2_small"), layers=3,
                               f_path=16, f_link=12, f_node=8, hidden=16, with_np=True)
    run_case(ref, "wide_L3", wide, synthetic_graph(wide, seed=2))
    # 128-wide features (the cfg2 row width), 2 layers
    w128 = dataclasses.replace(scaled_config(CONFIGS["cfg2"], 1e-3, name="cfg2_w128"),
                               f_path=128, f_link=128, f_node=128, hidden=128)
    run_case(ref, "w128_L2", w128, synthetic_graph(w128, seed=3))
    # two graphs collated PyG-style (offsets + batch vector), global feats + BatchNorm readout
    # (models.py:274-277 hard-codes global_feats_size = 8 = mean+max of a 4-wide path input, which the
    # 7/7/3 layout yields only with DIVIDED_FEATURES=false, BL_FEATURES=true: models.py:334-335)
    cfg1bl = dataclasses.replace(cfg1, bl_features=True)
    run_case(ref, "collate2_global_bn", cfg1bl, collate([synthetic_graph(cfg1bl, seed=4),
                                                         synthetic_graph(cfg1bl, seed=5)]),
             mlp_bn=True, global_feats=True)
    print("wrote fixtures to", HERE)


if __name__ == "__main__":
    main()
