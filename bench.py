"""Benchmark: HetroGIN training steps on MI355X (BASELINE.json metric), one process per GPU.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config cfg3]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

A step is one train.py iteration (train.py:31-44) on a resident synthetic hetero graph: zero_grad,
forward through every relation of every layer (as PyG computes them), sqrt(MAPE), backward, the RCCL
gradient all-reduce (N > 1), Adam.

Workload (default ``--config cfg3``, BASELINE.json configs[2]: 3 layers, 10M nodes / 100M edges, hidden 256,
fp32 — the graph the north star's >= 60 %-of-HBM aggregate target is stated on):
  * N = 1: the connected cfg3 graph (uniform endpoints over all 10M nodes).
  * N > 1: cfg4 (BASELINE configs[3]) — the same 100M edges generated as 8 independent
    components, each rank holding 8/N of them; the ranks train as ONE batch (hgin/dist.py: the gradient is
    that of sqrt(mape) over all paths).  Total work is fixed as N grows: "strong" scaling.
  ``--config cfg4`` runs the 8-component graph at N = 1 too (the 1-GPU point of the cfg4 curve); ``cfg5`` is
  cfg3 in bf16 (configs[4]); ``cfg2`` is configs[1].
  ``--partition dst-range`` (reported, not the headline): the connected graph itself over N ranks, each owning
  1/N of every node type's rows and the edges into them; per layer the source embeddings are all-gathered and
  their gradients reduce-scattered over RCCL (hgin/partition.py).

value = E_conv(total) / t_step, E_conv = edges of the four convolved relations (p->l, l->p, l->n, n->l),
counted once per step.  t_step = max over ranks of (barrier + hipDeviceSynchronize
bracketed K steps) / K (the bench contract); the median of the K per-step durations (HIP events between
steps on the step's stream) is reported beside it.  N > 1 (components): after the timed region
rank 0 alone also trains all the components the ranks split (2 warm-up + median of 5) and reports
``scaling_vs_1gpu`` = that step time / this run's median step (ideal N).  The timed region runs no probes: the
per-kernel HIP-event figures (``roofline``, ``gemm``) come from a separate untimed pass over the same step.

Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import ctypes
import dataclasses
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (ROOT, os.path.join(ROOT, "gnn-link-prediction_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = json.load(open(os.path.join(ROOT, "BASELINE.json")))["metric"]
HBM_PEAK_GBS = 8000.0        # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
F32_MFMA_PEAK_TFS = 157.3    # v_mfma_f32_32x32x2_f32 dense peak (= f32 vector peak)
BF16_MFMA_PEAK_TFS = 2500.0  # v_mfma_f32_32x32x16_bf16 dense peak (no sparsity)
# what a bare bf16 MFMA loop sustains on random operands once the chip lowers its clock under load (MI355X_MICROARCH.md
# "DVFS give-back" (1): 1,247 TF/s at 1.90-1.95 GHz; the 2.5 PF peak assumes 2.4 GHz) — reported beside the peak
BF16_MFMA_RANDOM_TFS = 1247.0
CPU_SAMPLE_EDGES = 1_000_000  # convolved edges of the bounded CPU-baseline sample (~10-30 s of CPU work)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="cfg3",
                    help="cfg3 (default, BASELINE configs[2]; N > 1: cfg4's 8-component split), cfg4, cfg5 (bf16), "
                         "cfg2, cfg2bf (bf16 at cfg2 size)")
    ap.add_argument("--partition", choices=("auto", "connected", "components", "dst-range"), default="auto",
                    help="auto: connected graph at N = 1 (cfg4: components), 8 components split over the ranks "
                         "at N > 1; dst-range: the connected graph with destination rows split over the ranks "
                         "(SURVEY.md §8.E connected-graph variant: per-layer all-gather / reduce-scatter)")
    ap.add_argument("--skew", choices=("uniform", "zipf"), default="uniform",
                    help="zipf: destination ids ~ Zipf(1.1) (SURVEY.md §8.D skew variant)")
    ap.add_argument("--prune-dead", action="store_true", help="skip dead relations (reported separately)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-probe", action="store_true", help="skip the untimed per-kernel event pass")
    ap.add_argument("--no-extras", action="store_true", help="skip the sampler / decoder / CSR-build lines")
    ap.add_argument("--no-ref1", action="store_true",
                    help="N > 1 components split: skip rank 0's single-GPU run of all the components (scaling_vs_1gpu)")
    ap.add_argument("--adam", choices=("foreach", "fused"), default="foreach",
                    help="torch.optim.Adam implementation (train.py's optimizer, same update rule)")
    ap.add_argument("--no-cfg5", action="store_true",
                    help="cfg3 at N = 1: skip the bf16 twin (BASELINE configs[4]) timed after the headline as extras.cfg5")
    ap.add_argument("--cpu-full", default=None, metavar="CFG",
                    help="only time the CPU baseline (oracle) on the FULL named config (e.g. cfg2) and print its record")
    ap.add_argument("--cpu-warmup", type=int, default=2, help="--cpu-full: warm-up steps (default 2)")
    ap.add_argument("--cpu-steps", type=int, default=5, help="--cpu-full: timed steps, median reported (default 5)")
    ap.add_argument("--graph", action="store_true",
                    help="one hipGraph replay per step (default: the step issued from Python; measured equal on cfg2 "
                         "and cfg5 — the step is GPU-bound, the host runs ahead)")
    ap.add_argument("--launch-dry-run", action="store_true",
                    help="print the rank-launch decision for --gpus as JSON and exit (touches no GPU)")
    return ap.parse_args()


def launch_plan(gpus: int, env, n_devices: int) -> dict:
    """How this invocation becomes `gpus` ranks (one process per GPU), decided before any HIP call.

    * WORLD_SIZE set (torch.distributed.run started us): it must equal --gpus, otherwise the line would report a
      different GPU count than asked for -> error.
    * --gpus N > 1 without WORLD_SIZE: re-launch through torch.distributed.run as N fresh child ranks (a child
      process, never an exec of this one), provided the node has N devices -> "spawn"; else error.
    * --gpus 1 without WORLD_SIZE: run here.
    HGIN_DIST_BACKEND=gloo is the 1-GPU rehearsal of the multi-rank path (ranks share the device), so the device
    count is not checked for it.  ``n_devices`` is torch.cuda.device_count(), which does not initialise HIP."""
    gloo = env.get("HGIN_DIST_BACKEND", "nccl") == "gloo"
    if gpus < 1:
        return {"action": "error", "reason": f"--gpus {gpus}: need at least one GPU"}
    ws = env.get("WORLD_SIZE")
    if ws is not None:
        if not ws.isdigit() or int(ws) != gpus:
            return {"action": "error",
                    "reason": f"--gpus {gpus} but the launcher set WORLD_SIZE={ws}: refusing to report a run of "
                              f"{ws} rank(s) as {gpus} GPU(s)"}
        return {"action": "run", "world": gpus}
    if gpus == 1:
        return {"action": "run", "world": 1}
    if n_devices < gpus and not gloo:
        return {"action": "error", "reason": f"--gpus {gpus} but this node shows {n_devices} GPU(s)"}
    return {"action": "spawn", "world": gpus,
            "argv": [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
                     "--master-addr", "127.0.0.1", "--master-port", "{port}", os.path.abspath(__file__)]}


def _free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def apply_launch_plan(args) -> None:
    """Carry out launch_plan before anything touches the GPU: exit non-zero on an error, or run the ranks as a child
    torch.distributed.run and exit with its status."""
    plan = launch_plan(args.gpus, os.environ, torch.cuda.device_count())
    if args.launch_dry_run:
        print(json.dumps(plan), flush=True)
        raise SystemExit(0)
    if plan["action"] == "error":
        print(f"bench.py: {plan['reason']}", file=sys.stderr, flush=True)
        raise SystemExit(2)
    if plan["action"] == "spawn":
        import subprocess
        argv = [a.replace("{port}", str(_free_port())) for a in plan["argv"]] + sys.argv[1:]
        print(f"bench.py: --gpus {args.gpus} without a launcher: starting {args.gpus} ranks via torch.distributed.run",
              file=sys.stderr, flush=True)
        raise SystemExit(subprocess.run(argv, env=dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")).returncode)


def cpu_threads() -> int:
    n = len(os.sched_getaffinity(0))
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        n = min(n, int(env))
    return max(1, n)


def host_ram_gb() -> float:
    try:
        for line in open("/proc/meminfo"):
            if line.startswith("MemTotal:"):
                return round(int(line.split()[1]) / 2 ** 20, 1)
    except OSError:
        pass
    return 0.0


def cpu_baseline(cfg, full_graph: bool = False, warmup: int = 2, steps: int = 5, progress: bool = False) -> dict:
    """The oracle (torch CPU ops == the PyG CPU path) on a bounded sample of the same workload, on this box's
    host cores: 2 warm-up steps, then the median of 5.  full_graph: the whole config instead of
    the ~1M-edge sample (cfg1 and cfg2 in full; a separate ``--cpu-full`` run, not the default
    bench line)."""
    from hgin.data import scaled_config, synthetic_graph
    from oracle.pyg_cpu import OracleHetroGIN, train_step
    threads = cpu_threads()
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    full = cfg
    # same schema and widths, every count scaled to ~1M convolved edges (the rate is per edge)
    if cfg.conv_edges > CPU_SAMPLE_EDGES and not full_graph:
        cfg = scaled_config(cfg, CPU_SAMPLE_EDGES / cfg.conv_edges, name=f"{cfg.name}-cpu-sample")
    # the reference's CPU path is fp32 only: a bf16 config is timed on its fp32 counterpart
    cfg = dataclasses.replace(cfg, feat_dtype="f32", components=1)
    times = []
    beat = None
    if progress:   # a full cfg3 step takes minutes: a heartbeat line every 30 s keeps the run visibly alive
        import threading
        stop = threading.Event()
        t_start = time.perf_counter()

        def _beat():
            while not stop.wait(30.0):
                print(f"cpu_baseline: {time.perf_counter() - t_start:.0f} s", file=sys.stderr, flush=True)
        beat = threading.Thread(target=_beat, daemon=True)
        beat.start()
    try:
        g = synthetic_graph(cfg, seed=0, device="cpu")
        torch.manual_seed(1997)
        model = OracleHetroGIN(**cfg.model_kwargs({"link": cfg.f_link, "path": cfg.f_path, "node": cfg.f_node}))
        opt = torch.optim.Adam(lr=1e-3, params=model.parameters())
        for i in range(warmup + steps):
            t0 = time.perf_counter()
            train_step(model, opt, g.x_dict(), g.edge_index_dict(), g.batch["path"], g.y)
            dt_i = time.perf_counter() - t0
            if i >= warmup:
                times.append(dt_i)
            if progress:
                print(json.dumps({"cpu_step": i, "warmup": i < warmup, "s": round(dt_i, 3),
                                  "loadavg_1m": round(os.getloadavg()[0], 1)}), file=sys.stderr, flush=True)
    finally:
        torch.set_num_threads(prev)
        if beat is not None:
            stop.set()
    dt = statistics.median(times)
    cpu_model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu_model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"value": round(cfg.conv_edges / dt, 1), "unit": "edges/s", "cores": threads, "kind": "port",
            "sample": f"{cfg.name}{' full graph' if cfg.nodes == full.nodes else ''} ({cfg.nodes} nodes / "
                      f"{cfg.graph_edges} edges, {cfg.conv_edges} convolved, hidden {cfg.hidden}, {cfg.layers} "
                      f"layers, fp32), {warmup} warm-up + median of {steps} train steps (fwd + sqrt-MAPE + bwd + Adam) of "
                      f"oracle/pyg_cpu.py (torch CPU ops = the reference's PyG CPU path), {threads} threads, "
                      f"{cpu_model}",
            "ms_per_step": round(dt * 1e3, 2), "host_ram_gb": host_ram_gb(),
            "step_times_s": [round(t, 3) for t in times],
            # the box's host is shared with other tenants' jobs: its load when the sample ran (1-minute average over
            # all of the machine's CPUs) says how contended the 16 threads were (DESIGN.md §5 CPU baseline)
            "host_loadavg_1m": round(os.getloadavg()[0], 1), "host_cpus": os.cpu_count()}


def zipf_dst(cfg, graph, dev, s: float = 1.1, seed: int = 7):
    """Skew variant: the forward relations' destination ids drawn from Zipf(s) over a random
    permutation of the destination type (reverse relations stay exact flips)."""
    from hgin.data import REL_LN, REL_LP, REL_NL, REL_PL, REL_PN
    g = torch.Generator(device=dev).manual_seed(seed)

    def draw(n_dst, n):
        ranks = torch.arange(1, n_dst + 1, device=dev, dtype=torch.float64)
        p = ranks.pow(-s)
        idx = torch.multinomial((p / p.sum()).float(), n, replacement=True, generator=g) if n_dst < 2 ** 24 else None
        if idx is None:
            raise ValueError("zipf: destination type too large for multinomial")
        perm = torch.randperm(n_dst, device=dev, generator=g)
        return perm[idx]

    ei = dict(graph.edge_index)
    for fwd, rev, n_dst in ((REL_PL, REL_LP, cfg.n_link), (REL_LN, REL_NL, cfg.n_node), (REL_PN, None, cfg.n_node)):
        if fwd not in ei:
            continue
        e = ei[fwd].clone()
        e[1] = draw(n_dst, e.size(1))
        ei[fwd] = e
        if rev is not None:
            ei[rev] = e.flip(0).contiguous()
    return dataclasses.replace(graph, edge_index=ei)


def csr_build_ms(graph, dev) -> dict:
    """CSR (by dst) + CSC (by src) build per convolved relation from scratch, HIP events (reported, not in
    t_step).  One untimed build of the first relation first, so the first timed build does not carry the
    sort kernels' one-time load / workspace allocation."""
    from hgin import ops
    from hgin.data import CONV_RELATIONS
    out = {}
    e0 = graph.edge_index[CONV_RELATIONS[0]]
    warm = ops.build_csr(e0, 1, graph.num_nodes(CONV_RELATIONS[0][2]), graph.num_nodes(CONV_RELATIONS[0][0]),
                         validate=False)
    torch.cuda.synchronize()
    del warm
    for rel in CONV_RELATIONS:
        e = graph.edge_index[rel]
        n_src, n_dst = graph.num_nodes(rel[0]), graph.num_nodes(rel[2])
        s, m, t = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        s.record()
        csr = ops.build_csr(e, 1, n_dst, n_src, validate=False)
        m.record()
        csc = ops.build_csr(e, 0, n_src, n_dst, validate=False)
        t.record()
        torch.cuda.synchronize()
        out["__".join(rel)] = {"edges": int(e.size(1)), "csr_ms": round(s.elapsed_time(m), 3),
                               "csc_ms": round(m.elapsed_time(t), 3)}
        del csr, csc
    return out


def one_gpu_reference(cfg, n_comp: int, dev, adam: str, graph_mode: bool, warmup: int = 2, steps: int = 5) -> dict:
    """The 1-GPU point of the strong-scaling curve measured inside an N > 1 run: rank 0 alone trains ALL n_comp
    components (the graph the N ranks split) on its GPU, a fresh model from the same seed, in the timed run's
    execution mode (eager, or one hipGraph replay per step with ``--graph``), 2 warm-up steps + the median of 5
    HIP-event-timed steps; the other ranks wait at a barrier."""
    from hgin import HetroGIN
    from hgin.data import rank_components
    from hgin.graphs import CapturedStaticStep
    from hgin.train import train_step
    graph, _ = rank_components(cfg, 0, 1, device=dev, n_components=n_comp)
    torch.manual_seed(1997)
    model = HetroGIN(**cfg.model_kwargs({"link": cfg.f_link, "path": cfg.f_path, "node": cfg.f_node})).to(dev)
    opt = torch.optim.Adam(lr=1e-3, params=model.parameters(), capturable=graph_mode,
                           **({"fused": True} if adam == "fused" else {}))
    if graph_mode:
        stepper = CapturedStaticStep(model, opt, graph, warmup=warmup)
        step = stepper.step
    else:
        step = lambda: train_step(model, opt, graph)  # noqa: E731
        for _ in range(warmup):
            step()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)]
    torch.cuda.synchronize()
    ev[0].record()
    for i in range(steps):
        step()
        ev[i + 1].record()
    torch.cuda.synchronize()
    ms = statistics.median(ev[i].elapsed_time(ev[i + 1]) for i in range(steps))
    del graph, model, opt, step
    torch.cuda.empty_cache()
    return {"ms_per_step_median": round(ms, 4), "components": n_comp, "warmup": warmup, "steps": steps,
            "execution": "hipgraph (one replay per step)" if graph_mode else "eager",
            "what": "rank 0 alone, all components of the split graph, after the timed region"}


def batches_extra(dev, n_graphs: int = 256, batch: int = 8, warmup: int = 5, steps: int = 200,
                  cfg_steps: int = 40) -> dict:
    """The reference's actual training loop (dataset.py:26, :239-244, train.py:25-44): shuffled
    batches of 8 small graphs.  Here: a cfg1-schema GraphStore (n_graphs RouteNet-sized graphs, 0.5x-1.5x cfg1,
    the reference's always-on normalisation applied once at build); each step = one device collation launch
    (GraphStore.collate_into) + one hipGraph replay of the whole train step: the fused small-batch step
    (hgin/smallbatch.py: 3 L + 1 kernels, Adam folded in) — the main figure whenever it takes config.json's model — and
    the general per-op path (hgin/graphs.py CapturedTrainStep) beside it.  ``configs``: the reference's other model
    switches (models.py / config.json) that the fused step refuses, each timed on the same batches through the path
    that takes it — MLP_BN, GLOBAL_FEATS, DROPOUT > 0, NODE_EMBEDDING_SIZE 128 and MODEL = "GAT" (HEADS 16,
    config.json's hidden 8 and 1 layer): all through the fused step now (HetroGAT included), the captured general path
    for what it refuses.  HIP events around the timed batches; reported beside the headline."""
    import numpy as np

    from hgin import HetroGAT, HetroGIN
    from hgin.data import CONFIGS, CONV_RELATIONS, scaled_config, synthetic_graph
    from hgin.graphs import CapturedTrainStep
    from hgin.smallbatch import SmallBatchStep
    from hgin.store import GraphStore
    from hgin.train import train_step
    base = CONFIGS["cfg1"]
    rng = np.random.default_rng(0)
    graphs = [synthetic_graph(scaled_config(base, float(rng.uniform(0.5, 1.5)), name=f"g{i}"), seed=i)
              for i in range(n_graphs)]
    store = GraphStore.build(graphs, device=dev, normalize=True)
    order = [rng.choice(n_graphs, batch, replace=False).tolist() for _ in range(warmup + steps)]
    conv_edges = [sum(int(store.edge_off[r][g + 1] - store.edge_off[r][g]) for r in CONV_RELATIONS for g in ids)
                  for ids in order[warmup:]]
    ic = lambda: {"link": base.f_link, "path": base.f_path, "node": base.f_node}   # noqa: E731

    def build(overrides=None, gat=False):
        torch.manual_seed(1997)
        kw = base.model_kwargs(ic())
        kw.update(overrides or {})
        if gat:
            kw = dict(kw, heads=16, node_embedding_size=8, message_passing_layers=1)
            return HetroGAT(**kw).to(dev)
        return HetroGIN(**kw).to(dev)

    def run(kind, model, n_steps):
        # the fused step folds Adam into its final kernel (SmallBatchStep(fold_optimizer=True)); the other paths run
        # torch's foreach Adam (measured faster there than fused Adam: 0.70 vs 0.90 ms per batch, profiles/r04/gpu_e)
        opt = torch.optim.Adam(lr=1e-3, params=model.parameters(), capturable=kind != "eager")
        seq = order[warmup:warmup + n_steps]
        if kind == "fused":
            stepper = SmallBatchStep(model, opt, store, batch, warmup_ids=order[:warmup], warmup=warmup)
            step = stepper.step
        elif kind == "captured":
            stepper = CapturedTrainStep(model, opt, store, batch, warmup_ids=order[:warmup], warmup=warmup)
            step = stepper.step
        else:   # eager exact batches: collation + every launch from the host per batch
            step = lambda ids: train_step(model, opt, store.collate(ids))   # noqa: E731
            for ids in order[:warmup]:
                step(ids)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        s.record()
        for ids in seq:
            loss = step(ids)
        e.record()
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / n_steps
        return {"ms_per_batch": round(s.elapsed_time(e) / n_steps, 4), "host_ms_per_batch": round(wall * 1e3, 4),
                "final_loss": float(loss), "batches": n_steps}

    exec_desc = {"fused": "the fused small-batch step (3 L + 1 kernels, Adam folded into the last) as one hipGraph "
                          "replay",
                 "captured": "per-op HIP kernels as one hipGraph replay (hgin/graphs.py CapturedTrainStep)",
                 "eager": "eager per-op HIP kernels on exact batches (store.collate + train_step)"}
    fused_ok = SmallBatchStep.supports(build())
    res, fused_error = {"general": run("captured", build(), steps)}, None
    if fused_ok:
        try:
            res["fused"] = run("fused", build(), steps)
        except Exception as exc:   # reported in the line, not fatal to the headline
            fused_error = f"{type(exc).__name__}: {exc}"[:300]
    main_kind = "fused" if "fused" in res else "general"
    m = res[main_kind]
    out = {"workload": f"{n_graphs} cfg1-schema graphs (7/7/3 raw features, normalised; sizes 0.5x-1.5x of "
                       f"{base.nodes} nodes / {base.graph_edges} edges) resident, shuffled batches of {batch}, "
                       f"hidden {base.hidden}, {base.layers} layers, fp32 (config.json's model)",
           "execution": "device collation (one batched-copy launch) + " + exec_desc[
               "fused" if main_kind == "fused" else "captured"],
           "batches": steps, "ms_per_batch": m["ms_per_batch"], "host_ms_per_batch": m["host_ms_per_batch"],
           "graphs_per_s": round(batch / (m["ms_per_batch"] / 1e3), 1),
           "edges_per_s": round(float(np.mean(conv_edges)) / (m["ms_per_batch"] / 1e3), 1),
           "mean_conv_edges_per_batch": float(np.mean(conv_edges)), "final_loss": m["final_loss"],
           "optimizer": ("torch.optim.Adam(lr=1e-3) folded into the fused step's final kernel" if main_kind == "fused"
                         else "torch.optim.Adam(lr=1e-3, capturable=True) (foreach)")}
    if main_kind == "fused":
        g = res["general"]
        out["general_path"] = dict(g, execution=exec_desc["captured"],
                                   optimizer="torch.optim.Adam(lr=1e-3, capturable=True) (foreach)")
    # the reference's other switches, each through the path that takes it (SmallBatchStep.supports says which)
    # (GLOBAL_FEATS needs BL_FEATURES: models.py:293 sizes the readout for [mean | max] of 4 path columns, which only
    # the bl_features slicing keeps, models.py:333-342 — with 3 columns the reference's own Linear raises)
    switches = {"mlp_bn": ({"mlp_bn": True}, False, "captured"),
                "global_feats": ({"global_feats": True, "bl_features": True}, False, "captured"),
                "dropout_0.1": ({"dropout": 0.1}, False, "captured"),
                "hidden_128": ({"node_embedding_size": 128}, False, "captured"),
                "gat_heads16_h8_L1": ({}, True, "captured")}
    cfgs = {}
    for name, (ov, gat, kind) in switches.items():
        try:
            model = build(ov, gat)
            if SmallBatchStep.supports(model):   # (HetroGAT too: k_sb_gat_fwd / k_sb_gat_bwd)
                kind = "fused"
            r = run(kind, model, cfg_steps)
            r["execution"] = exec_desc[kind]
            r["fused_step"] = "takes it" if kind == "fused" else "refuses it (SmallBatchStep.supports)"
            cfgs[name] = r
        except Exception as exc:   # reported, not fatal
            cfgs[name] = {"error": f"{type(exc).__name__}: {exc}"[:300]}
        torch.cuda.empty_cache()
    out["configs"] = cfgs
    # kernel-busy time per batch beside the event-timed figure: the step is a few short kernels, so the gap between
    # them (graph launch, dispatch) is a visible share of ms_per_batch.  Taken from the committed rocprofv3 kernel trace
    # of the same workload (tools/sb_prof.py -> tools/sb_busy.py), not measured in this run.
    for label, tgt in (("gin", out if main_kind == "fused" else None), ("gat", cfgs.get("gat_heads16_h8_L1"))):
        path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "r06", f"sb_busy_{label}.json")
        if tgt is not None and tgt.get("execution") != exec_desc["captured"] and os.path.exists(path):
            with open(path) as f:
                busy = json.load(f)
            tgt["kernel_ms_per_batch"] = busy["kernel_ms_per_batch"]
            tgt["kernel_trace"] = {"file": os.path.relpath(path, os.path.dirname(os.path.abspath(__file__))),
                                   "wall_ms_per_batch": busy["wall_ms_per_batch"],
                                   "launches_per_batch": busy["launches_per_batch"]}
    # the evaluation loops (train.py:70-113 test() after model.eval(), :322-348 evaluate()): config.json's
    # VAL_BATCH_SIZE 1, and the training batch size, as captured replays (hgin/graphs.py CapturedEvalStep: device
    # accumulators, one host sync per pass) beside the reference's eager form (forward + loss.item() per batch)
    from hgin.graphs import CapturedEvalStep
    from hgin.smallbatch import SmallBatchEval
    from hgin.train import mape as mape_fn
    ev = {}

    def eval_loop(model, bs, key, captured=True):
        seq = [order[warmup + i][:bs] for i in range(cfg_steps)]
        try:
            ev[key] = {"batches": cfg_steps}
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            if captured:
                st = CapturedEvalStep(model, store, bs, warmup_ids=[ids[:bs] for ids in order[:warmup]], warmup=2)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                s.record()
                for ids in seq:
                    st.step(ids)
                e.record()
                avg, _ = st.result(1)
                wall_c = (time.perf_counter() - t0) / cfg_steps
                ev[key].update(captured_ms_per_batch=round(s.elapsed_time(e) / cfg_steps, 4),
                               captured_host_ms_per_batch=round(wall_c * 1e3, 4), avg_loss=avg)
                del st
            t0 = time.perf_counter()
            tot = 0.0
            with torch.no_grad():
                for ids in seq:
                    b = store.collate(ids)
                    tot += float(mape_fn(model(b.x_dict(), b.edge_index_dict(), b.batch["path"]), b.y.reshape(-1, 1)))
            ev[key]["eager_host_ms_per_batch"] = round((time.perf_counter() - t0) / cfg_steps * 1e3, 4)
            ev[key]["eager_avg_loss"] = tot / cfg_steps
            if SmallBatchEval.supports(model):   # the fused kernels' forward (hgin/smallbatch.py SmallBatchEval)
                fe = SmallBatchEval(model, store, bs, warmup_ids=[ids[:bs] for ids in order[:warmup]], warmup=2)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                s.record()
                for ids in seq:
                    fe.step(ids)
                e.record()
                favg, _ = fe.result(1)
                wall_f = (time.perf_counter() - t0) / cfg_steps
                ev[key].update(fused_ms_per_batch=round(s.elapsed_time(e) / cfg_steps, 4),
                               fused_host_ms_per_batch=round(wall_f * 1e3, 4), fused_avg_loss=favg)
                del fe
        except Exception as exc:   # reported, not fatal
            ev[key] = {"error": f"{type(exc).__name__}: {exc}"[:300]}

    model = build()
    model.eval()
    for bs in (1, batch):
        eval_loop(model, bs, f"batch_{bs}")
    # HetroGAT's evaluation (train.py:120-125 MODEL == "GAT", config.json HEADS 16 x 8, 1 layer): fused and eager (the
    # captured padded path refuses GATConv's bipartite self loops, hgin/graphs.py _check_no_bipartite_loops)
    model = build(gat=True)
    model.eval()
    for bs in (1, batch):
        eval_loop(model, bs, f"gat_batch_{bs}", captured=False)
    del model
    out["eval"] = dict(ev, execution="captured: one batched-copy launch + one hipGraph replay (forward + fused head / "
                                     "MAPE + device accumulation) per batch; fused: the same around the small-batch "
                                     "kernels' forward (L + 2 launches; HetroGAT: 1 + 2); eager: collation + forward + "
                                     "loss.item() per batch, as train.py's test() / evaluate()")
    if fused_error:
        out["fused_path_error"] = fused_error
    return out


def gat_extra(dev, n_src: int = 6_000_000, n_dst: int = 3_000_000, E: int = 30_000_000, heads: int = 16, C: int = 8,
              reps: int = 5) -> dict:
    """HetroGAT's attention (models.py:413-418, PyG 2.0.2 GATConv; config.json HEADS 16 x hidden 8 = 128 columns) on
    one cfg3-sized relation (cfg3's p -> l shape: 6M sources, 3M destinations, 30M uniform edges + GATConv's self
    loops), after the headline: the forward attention kernel (hgin_gat_attn_fwd_f32, k_gat_attn_w: one pass, a_s formed
    from the gathered x_s rows) against HBM with its algorithmic bytes E'(4 + 4 H C + 4 H) + N_dst (8 + 4 H + 4 H C)
    (col, the gathered x_s row, the alpha store; rowptr, a_d, the output row), and the whole relation's attention
    forward + backward (logits, softmax-aggregate, destination- and source-side backward, att / bias column sums).
    HIP events, median of `reps`."""
    from hgin import _lib
    from hgin.gat import _GatAttentionFn, _logits, gat_graph
    from hgin.ops import _p, _stream
    g = torch.Generator(device=dev).manual_seed(7)
    HC = heads * C
    ei = torch.stack([torch.randint(0, n_src, (E,), device=dev, generator=g),
                      torch.randint(0, n_dst, (E,), device=dev, generator=g)])
    xs = torch.randn(n_src, HC, device=dev, generator=g)
    xd = torch.randn(n_dst, HC, device=dev, generator=g)
    att_s = (0.3 * torch.randn(1, heads, C, device=dev, generator=g)).requires_grad_()
    att_d = (0.3 * torch.randn(1, heads, C, device=dev, generator=g)).requires_grad_()
    bias = torch.zeros(HC, device=dev, requires_grad=True)
    graph = gat_graph(ei, n_src, n_dst, True)
    Ep = graph.n_edges
    a_d = _logits(xd, att_d.detach().reshape(-1).contiguous(), heads, C)
    alpha = torch.empty(Ep, heads, device=dev)
    out = torch.empty(n_dst, HC, device=dev)
    kern = []

    att_flat = att_s.detach().reshape(-1).contiguous()

    def fwd():   # the forward attention as GATConv runs it (hgin/gat.py: the one-pass kernel, a_s from the x_s rows)
        _lib.call("hgin_gat_attn_fwd_f32", _p(graph.csr.rowptr), _p(graph.csr.col), n_dst, heads, C, _p(xs),
                  xs.stride(0), _p(att_flat), _p(a_d), ctypes.c_float(0.2), None, None, 0, _p(alpha), _p(out),
                  out.stride(0), _stream(xs))

    def timed(fn):
        fn()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(reps + 1)]
        torch.cuda.synchronize()
        ev[0].record()
        for i in range(reps):
            fn()
            ev[i + 1].record()
        torch.cuda.synchronize()
        return statistics.median(ev[i].elapsed_time(ev[i + 1]) for i in range(reps))

    with _lib.trace_launches() as tr:
        fwd()
        torch.cuda.synchronize()
    kern = sorted(set(tr.kernels))
    f_ms = timed(fwd)
    algo = Ep * (4 + 4 * HC + 4 * heads) + n_dst * (8 + 4 * heads + 4 * HC)
    xs_g, xd_g = xs.requires_grad_(), xd.requires_grad_()
    g_out = torch.randn(n_dst, HC, device=dev, generator=g)

    def fwd_bwd():
        o = _GatAttentionFn.apply(xs_g, xd_g, att_s, att_d, bias, None, graph, heads, C, 0.2)
        o.backward(g_out)
    fb_ms = timed(fwd_bwd)
    achieved = algo / (f_ms / 1e3) / 1e9
    res = {"workload": f"one relation: {n_src} sources -> {n_dst} destinations, {E} uniform edges + self loops = {Ep} "
                       f"(GATConv's bipartite self-loop handling), heads {heads} x {C} = {HC} fp32 columns",
           "kernel": ",".join(kern), "fwd_attention_ms": round(f_ms, 4),
           "fwd_roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                            "frac": round(achieved / HBM_PEAK_GBS, 4), "bytes_per_launch": algo},
           "fwd_bwd_attention_ms": round(fb_ms, 4),
           "edges_per_s_fwd_bwd": round(Ep / (fb_ms / 1e3), 1),
           "timing": "HIP events, median of %d launches after one untimed" % reps}
    del ei, xs, xd, graph, alpha, out, g_out, xs_g, xd_g
    torch.cuda.empty_cache()
    return res


def extras(graph, dev) -> dict:
    """A10 / A11 throughput on the p->l relation's shapes (NOT IN REFERENCE rows; HIP events, 3 launches each)."""
    from hgin import linkpred
    from hgin.data import REL_PL
    e = graph.edge_index[REL_PL]
    n_dst = graph.num_nodes("link")
    k = 4
    n = int(e.size(1)) * k
    res = {}

    def timed(fn, reps=3):
        fn()
        s, t = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            fn()
        t.record()
        torch.cuda.synchronize()
        return s.elapsed_time(t) / reps

    ms = timed(lambda: linkpred.sample_negative_dst(n, n_dst, seed=1, device=dev))
    res["neg_sample"] = {"samples": n, "ms": round(ms, 4), "bytes": 4 * n,
                         "GB_s": round(4 * n / (ms / 1e3) / 1e9, 1),
                         "frac_hbm": round(4 * n / (ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4)}
    zs, zd = graph.x["path"], graph.x["link"]
    if zs.dtype == torch.float32 and zs.size(1) == zd.size(1):
        from hgin import _lib, ops
        src32 = e[0].to(torch.int32)
        dst32 = e[1].to(torch.int32)
        score = torch.empty(e.size(1), dtype=torch.float32, device=dev)
        F = int(zs.size(1))
        E = int(e.size(1))

        def fwd():
            _lib.call("hgin_dot_decode_fwd_f32", ops._p(src32), ops._p(dst32), E, ops._p(zs), zs.stride(0),
                      ops._p(zd), zd.stride(0), F, ops._p(score), ops._stream(score))

        ms = timed(fwd)
        b = E * (2 * 4 + 2 * 4 * F + 4)
        res["dot_decode_fwd"] = {"pairs": E, "width": F, "ms": round(ms, 4), "bytes": b,
                                 "GB_s": round(b / (ms / 1e3) / 1e9, 1),
                                 "frac_hbm": round(b / (ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4)}
    return res


def cfg5_extra(dev, adam: str, warmup: int = 2, steps: int = 5) -> dict:
    """BASELINE configs[4] (cfg5: cfg3's graph and model with bf16 features + bf16 MFMA, fp32 accumulate) timed in the
    same run after the cfg3 headline has been freed: warm-up, then `steps` steps bracketed by hipDeviceSynchronize
    (wall) with HIP events per step, then an untimed probe pass for its aggregate roofline and GEMM families."""
    from hgin import HetroGIN, profiling
    from hgin.data import CONFIGS, synthetic_graph
    from hgin.train import train_step
    cfg = CONFIGS["cfg5"]
    graph = synthetic_graph(cfg, seed=0, device=dev)
    torch.manual_seed(1997)
    model = HetroGIN(**cfg.model_kwargs({"link": cfg.f_link, "path": cfg.f_path, "node": cfg.f_node})).to(dev)
    opt = torch.optim.Adam(lr=1e-3, params=model.parameters(), weight_decay=0,
                           **({"fused": True} if adam == "fused" else {}))
    for _ in range(warmup):
        train_step(model, opt, graph)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev[0].record()
    for i in range(steps):
        loss = train_step(model, opt, graph)
        ev[i + 1].record()
    torch.cuda.synchronize()
    t_step = (time.perf_counter() - t0) / steps
    t_med = statistics.median(ev[i].elapsed_time(ev[i + 1]) for i in range(steps)) / 1e3
    probe = profiling.start()
    for _ in range(2):
        train_step(model, opt, graph)
    profiling.stop()
    s = probe.summary()
    a = s.get("aggregate")
    roofline = None
    if a:
        achieved = a["avg_work"] / (a["avg_ms"] / 1e3) / 1e9
        roofline = {"bound": "hbm", "kernel": "hgin_aggregate_bf16 (k_agg_pipe: CSR forward + CSC backward)",
                    "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(achieved / HBM_PEAK_GBS, 4), "bytes_per_launch": a["avg_work"],
                    "avg_launch_ms": round(a["avg_ms"], 5), "launches_per_step": a["launches"] / 2}
    out = {"workload": f"cfg5 (BASELINE configs[4]): cfg3's {cfg.nodes} nodes / {cfg.graph_edges} edges, hidden "
                       f"{cfg.hidden}, {cfg.layers} layers, bf16 features + bf16 MFMA, fp32 accumulate, one GPU",
           "steps": steps, "warmup": warmup, "ms_per_step": round(t_step * 1e3, 4),
           "ms_per_step_median": round(t_med * 1e3, 4), "value": round(cfg.conv_edges / t_step, 1),
           "unit": "edges/s", "dtype": "bf16", "roofline": roofline,
           "gemm": gemm_fields(s.get("gin_mlp"), True, 2, t_step, "forward MLP GEMM (hgin_gin_mlp_fwd_bf16)"),
           "gemm_dw": gemm_fields(s.get("gemm_dw"), True, 2, t_step, "weight-gradient GEMMs (bf16)"),
           "gemm_dx": gemm_fields(s.get("gemm_dx"), True, 2, t_step, "input-gradient GEMMs (bf16)"),
           "final_loss": float(loss),
           "timing": "after the cfg3 headline's graph and model were freed; wall clock over the steps bracketed by "
                     "hipDeviceSynchronize, per-step HIP events for the median, separate probe pass"}
    del graph, model, opt, probe
    torch.cuda.empty_cache()
    return out


def traffic_file(name: str):
    """The newest committed PMC traffic record for this config (profiles/r*/traffic_<cfg>.json)."""
    import glob
    fs = sorted(glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]", f"traffic_{name}.json")))
    return fs[-1] if fs else None


def gemm_fields(m, bf16: bool, steps: int, t_step: float, what: str):
    """One GEMM family's roofline fields from the probe's HIP events over whole calls: HBM (algorithmic bytes
    / time) and the matrix cores (bf16-product FLOP/s / the 2.5 PFLOP/s dense bf16 peak; an fp32 multiply-add
    costs six bf16 products in the 3-way split, so its fp32-equivalent rate is a sixth of that)."""
    if not m:
        return None
    sec = m["avg_ms"] / 1e3
    gbs = m["avg_bytes"] / sec / 1e9
    tfs = m["avg_work"] / sec / 1e12
    # the fp32 GEMM mode libhgin.so runs (hgin_common.h gemm_split_enabled: the same process-static switch)
    mfma32 = not bf16 and os.environ.get("HGIN_F32_GEMM") == "mfma32"
    mode = "bf16" if bf16 else ("f32 MFMA (v_mfma_f32_32x32x2_f32)" if mfma32 else "fp32 as 3-way bf16 split, 6 products")
    products = 1 if (bf16 or mfma32) else 6
    peak = F32_MFMA_PEAK_TFS if mfma32 else BF16_MFMA_PEAK_TFS
    mfma = tfs * products
    hf, mf = gbs / HBM_PEAK_GBS, mfma / peak
    return {"kernel": what, "mode": mode, "bound": "hbm" if hf >= mf else "mfma",
            "hbm": {"achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(hf, 4)},
            "mfma": {"achieved": round(mfma, 1), "peak": peak,
                     "unit": "TFLOP/s (f32)" if mfma32 else "TFLOP/s (bf16 products)",
                     "frac": round(mf, 4), "products_per_fma": products,
                     "fp32_equivalent_tflops": None if bf16 else round(tfs, 2),
                     "random_operand_loop": None if mfma32 else {
                         "tflops": BF16_MFMA_RANDOM_TFS, "frac": round(mfma / BF16_MFMA_RANDOM_TFS, 4),
                         "source": "MI355X_MICROARCH.md DVFS give-back (1): bf16 MFMA loop, random operands, "
                                   "1.90-1.95 GHz"}},
            "bytes_per_launch": m["avg_bytes"], "flops_per_launch": m["avg_work"],
            "avg_launch_ms": round(m["avg_ms"], 5), "launches_per_step": m["launches"] / steps,
            "ms_per_step": round(m["total_ms"] / steps, 3),
            "share_of_step": round(m["total_ms"] / steps / (t_step * 1e3), 4)}


def main():
    args = parse()
    if not args.cpu_full:
        apply_launch_plan(args)
    if args.cpu_full:
        from hgin.data import CONFIGS
        rec = cpu_baseline(CONFIGS[args.cpu_full], full_graph=True, warmup=args.cpu_warmup, steps=args.cpu_steps,
                           progress=True)
        print(json.dumps({"cpu_baseline_full": args.cpu_full, **rec}), flush=True)
        return rec
    from hgin import HetroGIN, _lib, profiling
    from hgin.data import CONFIGS, rank_components, synthetic_graph
    from hgin.dist import GradAllReducer
    from hgin.graphs import CapturedStaticStep
    from hgin.partition import DstRangePartition
    from hgin.partition import train_step as partition_step
    from hgin.train import train_step

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    assert world == args.gpus, (world, args.gpus)   # apply_launch_plan guarantees it
    # One rank per GPU.  HGIN_DIST_BACKEND=gloo (+ more ranks than GPUs) is only for rehearsing the
    # multi-rank path on a 1-GPU box; the measured runs use RCCL ("nccl" on ROCm) over xGMI.
    backend = os.environ.get("HGIN_DIST_BACKEND", "nccl")
    dev = torch.device("cuda", local % max(torch.cuda.device_count(), 1))
    torch.cuda.set_device(dev)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    _lib.lib()

    cfg = CONFIGS[args.config]
    bf16 = cfg.feat_dtype == "bf16"
    mfma_peak = BF16_MFMA_PEAK_TFS if bf16 else F32_MFMA_PEAK_TFS
    partition = args.partition
    if partition == "auto":
        partition = "components" if (world > 1 or cfg.components > 1) else "connected"
    if partition == "components":
        n_comp = cfg.components if cfg.components > 1 else 8
        graph, comp_ids = rank_components(cfg, rank, world, device=dev, n_components=n_comp)
        total_conv_edges = cfg.conv_edges          # the ranks split one fixed graph
        scaling = "strong"
        part_desc = (f"{n_comp} independent components of {cfg.name}'s totals ({cfg.conv_edges // n_comp} convolved "
                     f"edges each), {len(comp_ids)} per rank")
    elif partition == "dst-range":
        full = synthetic_graph(cfg, seed=0, device=dev)
        if args.skew == "zipf":
            full = zipf_dst(cfg, full, dev)
        dst_part = DstRangePartition({t: full.num_nodes(t) for t in full.x})
        graph = dst_part.local_graph(full)
        del full
        comp_ids = [0]
        total_conv_edges = cfg.conv_edges
        scaling = "strong"
        elem = 2 if cfg.feat_dtype == "bf16" else 4
        widths0 = {"path": cfg.f_path, "link": cfg.f_link, "node": cfg.f_node}
        widths = {t: cfg.hidden for t in widths0}
        # forward: one all-gather per layer (the first of raw features, L - 1 of hidden embeddings); backward: one
        # reduce-scatter per layer above the first (the raw features need no gradient): 2L - 2 hidden rounds
        xchg = dst_part.exchange_bytes(widths0, elem) + (2 * cfg.layers - 2) * dst_part.exchange_bytes(widths, elem)
        part_desc = (f"one connected graph, destination rows of every node type split over {world} rank(s) "
                     f"(per-layer all-gather of source embeddings / reduce-scatter of their gradients, "
                     f"{xchg / 1e9:.2f} GB received per rank per step)")
    else:
        if world > 1:
            raise SystemExit("--partition connected: one connected graph per rank is not a data-parallel split of "
                             "one workload; use components or dst-range")
        graph = synthetic_graph(cfg, seed=0, device=dev)
        comp_ids = [0]
        total_conv_edges = cfg.conv_edges
        scaling = "strong"
        part_desc = "one connected graph"
    if args.skew == "zipf" and partition != "dst-range":
        graph = zipf_dst(cfg, graph, dev)
    torch.manual_seed(1997)
    model = HetroGIN(**cfg.model_kwargs({"link": cfg.f_link, "path": cfg.f_path, "node": cfg.f_node})).to(dev)
    if args.prune_dead:
        model.prune_dead(True)
    # capturable Adam: the optimizer step is part of the replayed graph (same update rule and arithmetic)
    opt = torch.optim.Adam(lr=1e-3, params=model.parameters(), weight_decay=0, capturable=args.graph,
                           **({"fused": True} if args.adam == "fused" else {}))
    reducer = GradAllReducer(model.parameters()) if (world > 1 or partition == "dst-range") else None
    stepper = None

    def barrier():
        if world > 1:
            dist.barrier(device_ids=[dev.index]) if backend == "nccl" else dist.barrier()

    # the dst-range graph is a rank's share (local destination ids, global source ids): no standalone extras
    no_extras = args.no_extras or partition == "dst-range"
    csr_ms = None
    if rank == 0 and not no_extras:
        csr_ms = csr_build_ms(graph, dev)     # separate cold builds; the model builds its own cached copies

    if partition == "dst-range":
        if args.graph:
            raise SystemExit("--graph: the dst-range partition's collectives run eagerly")
        eager_step = lambda: partition_step(model, opt, dst_part, graph, reducer=reducer)  # noqa: E731
    else:
        eager_step = lambda: train_step(model, opt, graph, reducer=reducer)  # noqa: E731
    if not args.graph:
        for _ in range(args.warmup):
            eager_step()
        step = eager_step
    else:
        # W eager warm-up steps, then the step is captured once and replayed once untimed
        stepper = CapturedStaticStep(model, opt, graph, reducer=reducer, warmup=args.warmup)
        stepper.step()
        step = stepper.step
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev[0].record()
    for i in range(args.steps):
        loss = step()
        ev[i + 1].record()
    torch.cuda.synchronize()
    barrier()
    t1 = time.perf_counter()
    per_step = [ev[i].elapsed_time(ev[i + 1]) for i in range(args.steps)]
    dt = torch.tensor([(t1 - t0) / args.steps, statistics.median(per_step) / 1e3], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(dt, op=dist.ReduceOp.MAX)
    t_step, t_med = float(dt[0].item()), float(dt[1].item())
    # every rank's peak device footprint over setup + warm-up + the timed steps (before the probe / reference passes)
    peak = torch.zeros(world, dtype=torch.float64, device=dev)
    peak[rank] = torch.cuda.max_memory_allocated(dev) / 1e9
    if world > 1:
        dist.all_reduce(peak)
    peak_per_rank = [round(float(v), 2) for v in peak.tolist()]
    final_loss = float(loss)
    if reducer is not None:
        reducer.check()   # one host sync after the timed region: every rank reduced the same parameter set

    # untimed per-kernel pass: the same eager step with HIP events around the aggregate and GEMM launches
    probe = None
    steps_recorded = min(args.steps, 3)
    if not args.no_probe:
        probe = profiling.start()
        for _ in range(steps_recorded):
            eager_step()
        profiling.stop()

    ref1 = None
    if world > 1 and partition == "components" and args.skew == "uniform" and not (args.no_ref1 or args.prune_dead):
        if rank == 0:
            ref1 = one_gpu_reference(cfg, n_comp, dev, args.adam, args.graph)
        barrier()

    extra = None
    if rank == 0 and not no_extras:
        extra = extras(graph, dev)
        try:
            extra["batches"] = batches_extra(dev)
        except Exception as exc:   # reported in the line, not fatal to the headline
            extra["batches"] = {"error": f"{type(exc).__name__}: {exc}"[:300]}
            torch.cuda.empty_cache()

    out = None
    if rank == 0:
        value = total_conv_edges / t_step
        roofline = gemm = gemm_dw = gemm_dx = None
        if probe is not None:
            s = probe.summary()
            a = s.get("aggregate")
            if a:
                achieved = a["avg_work"] / (a["avg_ms"] / 1e3) / 1e9
                roofline = {"bound": "hbm",
                            "kernel": ("hgin_aggregate_bf16 (k_agg_pipe: CSR forward + CSC backward)" if bf16 else
                                       "hgin_aggregate_f32 (k_aggregate: CSR forward + CSC backward)"),
                            "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
                            "bytes_per_launch": a["avg_work"], "avg_launch_ms": round(a["avg_ms"], 5),
                            "launches_per_step": a["launches"] / steps_recorded,
                            "share_of_step": round(a["total_ms"] / steps_recorded / (t_step * 1e3), 4),
                            "timing": "HIP events on the launching stream, untimed probe pass after the timed steps"}
                tf = traffic_file(cfg.name)
                if tf and partition == "connected" and args.skew == "uniform" and world == 1:
                    tr = json.load(open(tf))
                    roofline["traffic"] = tr.get("bytes_per_launch")
                    roofline["traffic_source"] = tr.get("source")
                    roofline["traffic_measured"] = (f"committed constant: PMC FETCH_SIZE / WRITE_SIZE passes of an "
                                                    f"earlier rocprofv3 run of this command "
                                                    f"({os.path.relpath(tf, ROOT)}), not counters of this run")
            gemm = gemm_fields(s.get("gin_mlp"), bf16, steps_recorded, t_step, "forward MLP GEMM "
                               f"(hgin_gin_mlp_fwd_{'bf16' if bf16 else 'f32'}: "
                               f"{'k_ws_bf16 / k_gemm_nt_bf16' if bf16 else 'k_wss_f32 / k_ws_f32 / k_gemm_nt'} + bias / PReLU / "
                               f"accum epilogue)")
            gemm_dw = gemm_fields(s.get("gemm_dw"), bf16, steps_recorded, t_step,
                                  "weight-gradient GEMMs (hgin_gin_mlp_bwd_w_* / hgin_gemm_tn_*, incl. the fused or "
                                  "separate PReLU backward and the slab sums)")
            gemm_dx = gemm_fields(s.get("gemm_dx"), bf16, steps_recorded, t_step,
                                  "input-gradient GEMMs (hgin_gemm_nt_combine_* / hgin_gemm_nt_*, incl. the "
                                  "self-term backward epilogue and its eps sum)")
        wl = (f"{cfg.name}: {cfg.layers}-layer HeteroGIN, {cfg.nodes} nodes / {cfg.graph_edges} edges total, 3 node "
              f"types x {len(graph.edge_index)} edge types, hidden {cfg.hidden} {'bf16' if bf16 else 'fp32'}, "
              f"{part_desc}" + (", dst ~ Zipf(1.1)" if args.skew == "zipf" else ""))
        out = {"metric": METRIC, "value": round(value, 1), "unit": "edges/s", "n_gpus": world,
               "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(t_step * 1e3, 4),
               "ms_per_step_median": round(t_med * 1e3, 4),
               "higher_is_better": True, "scaling": scaling, "vs_baseline": None,
               "dtype": "bf16" if bf16 else "f32", "accumulate": "f32",
               "data": "synthetic: SURVEY.md §8.D generator (uniform endpoints, reverse relations = flips, randn "
                       "features, rand+0.5 labels), random-init weights (seed 1997)",
               "config": {"workload": wl, "nodes": cfg.nodes, "graph_edges": cfg.graph_edges,
                          "conv_edges": total_conv_edges, "hidden": cfg.hidden, "layers": cfg.layers,
                          "partition": partition, "components_per_rank": len(comp_ids),
                          "global_batch": len(comp_ids) * world,
                          "parallelism": ("single GPU" if world == 1 else
                                          f"dst-range partition over {world} ranks: per-layer all-gather / "
                                          f"reduce-scatter of node embeddings + one all-reduce of gradients and "
                                          f"loss sums" if partition == "dst-range" else
                                          f"dp{world} over graph components, one RCCL all-reduce per step "
                                          f"(gradients + loss sums)"),
                          "world_size": world, "backend": (f"{backend} ({'RCCL' if backend == 'nccl' else backend})"
                                                           if world > 1 else None),
                          "skew": args.skew, "prune_dead": bool(args.prune_dead),
                          "execution": "hipgraph (one replay per step)" if args.graph else "eager",
                          "optimizer": f"torch.optim.Adam(lr=1e-3), {args.adam}"},
               "roofline": roofline, "gemm": gemm, "gemm_dw": gemm_dw, "gemm_dx": gemm_dx, "csr_build": csr_ms, "extras": extra, "final_loss": final_loss}
        if (world == 1 and cfg.name == "cfg3" and partition == "connected" and args.skew == "uniform" and
                not (no_extras or args.no_cfg5 or args.prune_dead or args.graph)):
            # BASELINE configs[4] in the same driver-run line: free the cfg3 graph / model first (60 + 35 GB)
            del graph, model, opt, step, eager_step, stepper, probe, reducer
            torch.cuda.synchronize()
            torch.cuda.empty_cache()
            out["extras"]["cfg5"] = cfg5_extra(dev, args.adam)
            try:   # a failing extra is reported in the line, never fatal to the headline
                out["extras"]["gat"] = gat_extra(dev)
            except Exception as exc:
                out["extras"]["gat"] = {"error": f"{type(exc).__name__}: {exc}"[:300]}
                torch.cuda.empty_cache()
        if ref1 is not None:
            # strong scaling against the same graph on one GPU: t_1gpu / t_step (ideal: N)
            out["one_gpu_reference"] = ref1
            out["scaling_vs_1gpu"] = round(ref1["ms_per_step_median"] / (t_med * 1e3), 3)
        # the worst-case device footprint of this rank: its share, rank 0's all-component reference and the extras
        out["peak_device_mem_gb"] = round(torch.cuda.max_memory_allocated(dev) / 1e9, 2)
        out["peak_device_mem_gb_timed_per_rank"] = peak_per_rank
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(cfg)
        else:
            out["cpu_baseline"] = None
        print(json.dumps(out), flush=True)
    if world > 1:
        barrier()
        dist.destroy_process_group()
    return out


if __name__ == "__main__":
    main()
