"""bf16 forward GIN GEMM at the first layer's K = 512 (cfg5): cost of the eps-scaled self half.  Times
hgin_gin_mlp_fwd_bf16 with A = [agg | (1 + eps) x_dst] (two sources, eps), [agg | x_dst] (two sources, no eps) and
one 512-wide source, M = 6M / 3M / 1M, N = 256."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gnn-link-prediction_amd")]

import torch  # noqa: E402

from hgin import _lib, ops  # noqa: E402


def timeit(fn, reps=10):
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
    g = torch.Generator(device="cuda").manual_seed(1)
    BF = torch.bfloat16
    for M in (6_000_000, 3_000_000, 1_000_000):
        a = torch.randn(M, 512, device="cuda", generator=g).to(BF)
        a1, a2 = a[:, :256].contiguous(), a[:, 256:].contiguous()
        w = (torch.randn(256, 512, device="cuda", generator=g) / 512 ** 0.5).to(BF)
        b = torch.randn(256, device="cuda", generator=g)
        s = torch.tensor([0.25], device="cuda")
        eps = torch.tensor([0.1], device="cuda")
        gb = 2 * M * (512 + 2 * 256) / 1e9
        for name, fn in (("two sources + eps", lambda: ops.gin_mlp_fwd(a1, w, b, s, None, comb2=a2, eps2=eps)),
                         ("two sources", lambda: ops.gin_mlp_fwd(a1, w, b, s, None, comb2=a2)),
                         ("one source", lambda: ops.gin_mlp_fwd(a, w, b, s, None))):
            with _lib.trace_launches() as tr:
                fn()
            t = timeit(fn)
            print(f"M={M} K=512 N=256 {name:18s}: {t:7.3f} ms {gb / t:6.2f} TB/s  {sorted(set(tr.kernels))}",
                  flush=True)
        del a, a1, a2
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
