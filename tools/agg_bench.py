"""Micro-benchmark of the fused aggregate kernel on the cfg2 / cfg3 relation shapes (algorithmic GB/s)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gnn-link-prediction_amd")]

import torch  # noqa: E402

from hgin import ops, profiling  # noqa: E402


def timeit(fn, reps=20):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    dt = torch.bfloat16 if "--bf16" in sys.argv else torch.float32
    g = torch.Generator(device="cuda").manual_seed(0)
    # (name, n_src, n_dst, E, F, mode)
    cases = [("p->l L0 concat", 600_000, 300_000, 3_000_000, 128, 2),
             ("l->p L0 concat", 300_000, 600_000, 3_000_000, 128, 2),
             ("l->p L1 add", 300_000, 600_000, 3_000_000, 128, 1),
             ("p->l bwd none", 600_000, 300_000, 3_000_000, 128, 0),
             ("cfg3 l->p concat", 3_000_000, 6_000_000, 30_000_000, 256, 2),
             ("cfg3 p->l add", 6_000_000, 3_000_000, 30_000_000, 256, 1),
             ("cfg3 l->p bwd none", 3_000_000, 6_000_000, 30_000_000, 256, 0)]
    for name, n_src, n_dst, E, F, mode in cases:
        ei = torch.stack([torch.randint(0, n_src, (E,), device="cuda", generator=g),
                          torch.randint(0, n_dst, (E,), device="cuda", generator=g)])
        graph = ops.relation_graph(ei, n_src, n_dst)
        x = torch.randn(n_src, F, device="cuda", generator=g).to(dt)
        xd = torch.randn(n_dst, F, device="cuda", generator=g).to(dt) if mode else None
        eps = torch.zeros(1, device="cuda") if mode else None
        out = torch.empty(n_dst, F * (2 if mode == 2 else 1), device="cuda", dtype=dt)
        t = sorted(timeit(lambda: ops.aggregate_into(graph.csr, x, xd, eps, mode, out)) for _ in range(3))[1]
        b = profiling.aggregate_bytes(E, n_dst, F, F if mode else 0, mode, x.element_size())
        print(f"{os.environ.get('HGIN_AGG_PIPE', '-')} {str(dt)[6:]:8s} {name:18s} {t * 1e3:8.1f} us  {b / 1e9:6.2f} GB  {b / (t / 1e3) / 1e9:7.0f} GB/s")
        del ei, graph, x, xd, out
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
