"""dX GEMM with the fused self-term backward (hgin_gemm_nt_combine_*) vs the plain dX GEMM followed by
hgin_combine_bwd_*, at the add-mode shapes of cfg2 (fp32) and cfg5 (bf16).  Interleaved rounds, median."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gnn-link-prediction_amd")]

import torch  # noqa: E402

from hgin import ops  # noqa: E402
from mlp_bwd_bench import timeit  # noqa: E402


def main():
    for dt, shapes in ((torch.float32, [(600_000, 128, 128), (300_000, 128, 128)]),
                       (torch.bfloat16, [(6_000_000, 256, 256), (3_000_000, 256, 256), (600_000, 128, 128)])):
        for M, H, F in shapes:
            gz = torch.randn(M, H, device="cuda").to(dt)
            wt = torch.randn(F, H, device="cuda").to(dt)
            xd = torch.randn(M, F, device="cuda").to(dt)
            eps = torch.tensor([0.1], device="cuda")

            def sep():
                c = ops.gemm_nt(gz, wt)
                ops.combine_bwd(c, xd, eps, True)

            cases = [("gemm_nt", lambda: ops.gemm_nt(gz, wt)), ("combine_bwd", lambda: ops.combine_bwd(gz, xd, eps, True)),
                     ("separate", sep), ("fused", lambda: ops.gemm_nt_combine(gz, wt, xd, eps, 0, True))]
            res = {}
            for _ in range(3):
                for name, fn in cases:
                    res.setdefault(name, []).append(timeit(fn, reps=10))
            print(f"M={M} H={H} F={F} {dt}: " + "  ".join(f"{n} {sorted(v)[1] * 1e3:.1f} us" for n, v in res.items()),
                  flush=True)
            del gz, wt, xd
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
