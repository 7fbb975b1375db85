"""Micro-benchmark of the MFMA GEMM kernels vs hipBLASLt (torch.mm) on the shapes of a cfg2/cfg3 step.
Interleaved rounds in one process (cdna_hip_programming.md §5.4 rule 24); median of the rounds."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gnn-link-prediction_amd")]

import torch  # noqa: E402

from hgin import ops  # noqa: E402


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
    shapes = [(600_000, 256, 128), (600_000, 128, 128), (300_000, 256, 128), (6_000_000 // 4, 512, 256),
              (1_500_000, 256, 256)]
    for a in sys.argv[1:]:
        if a.startswith("--shapes="):     # e.g. --shapes=300000x256x128,294912x256x128  (M x K x N)
            shapes = [tuple(int(v) for v in s.split("x")) for s in a.split("=", 1)[1].split(",")]
    for M, K, N in shapes:
        a = torch.randn(M, K, device="cuda")
        w = torch.randn(N, K, device="cuda") / K ** 0.5
        b = torch.randn(N, device="cuda")
        s = torch.tensor([0.25], device="cuda")
        acc = torch.randn(M, N, device="cuda")
        gz = torch.randn(M, N, device="cuda")
        flops = 2.0 * M * N * K
        res = {}
        quick = "--quick" in sys.argv
        for _ in range(3):
            for name, fn in ([("mlp_fwd(z,y,accum)", lambda: ops.gin_mlp_fwd(a, w, b, s, acc)),
                              ("gemm_nt", lambda: ops.gemm_nt(a, w)),
                              ("gemm_tn dW", lambda: ops.gemm_tn(gz, a))] if quick else [
                ("mlp_fwd(z,y,accum)", lambda: ops.gin_mlp_fwd(a, w, b, s, acc)),
                ("mlp_fwd(y only)", lambda: ops.gin_mlp_fwd(a, w, b, s, None, save_z=False)),
                ("gemm_nt", lambda: ops.gemm_nt(a, w)),
                ("torch.mm a@w^T", lambda: torch.mm(a, w.t())),
                ("gemm_tn dW", lambda: ops.gemm_tn(gz, a)),
                ("torch.mm gz^T@a", lambda: torch.mm(gz.t(), a)),
                ("gemm_nt dX", lambda: ops.gemm_nt(gz, w.t().contiguous())),
                ("torch.mm gz@w", lambda: torch.mm(gz, w)),
            ]):
                res.setdefault(name, []).append(timeit(fn))
        print(f"M={M} K={K} N={N}  ({flops / 1e9:.1f} GF)")
        for name, ts in res.items():
            t = sorted(ts)[len(ts) // 2]
            print(f"   {name:22s} {t * 1e3:9.1f} us  {flops / (t / 1e3) / 1e12:7.1f} TF/s")
        del a, w, acc, gz
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
