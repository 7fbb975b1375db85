"""fp32 forward MLP GEMM (hgin_gin_mlp_fwd_f32) at the cfg3 / cfg2 layer shapes: GB/s of its HBM bytes
(A read once, z and y written, accum read).  Run once per HGIN_NT_WS32 setting (the switch is process-static):

    python tools/ws32_bench.py            # k_ws_f32 (default)
    HGIN_NT_WS32=0 python tools/ws32_bench.py   # the tiled k_gemm_nt
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gnn-link-prediction_amd")]

import torch  # noqa: E402

from hgin import ops  # noqa: E402


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
    shapes = [(6_000_000, 256, 256, True), (3_000_000, 256, 256, False), (1_000_000, 256, 256, True),
              (600_000, 128, 128, True)]
    out = []
    for M, K, N, with_acc in shapes:
        a = torch.randn(M, K, device="cuda")
        w = torch.randn(N, K, device="cuda") / K ** 0.5
        b = torch.randn(N, device="cuda")
        s = torch.tensor([0.25], device="cuda")
        acc = torch.randn(M, N, device="cuda") if with_acc else None
        ms = timeit(lambda: ops.gin_mlp_fwd(a, w, b, s, acc, save_z=True))
        byt = 4.0 * (M * K + M * N * (2 + (1 if with_acc else 0)))
        out.append({"M": M, "K": K, "N": N, "accum": with_acc, "ms": round(ms, 4), "GB_s": round(byt / ms / 1e6, 1),
                    "tflops_equiv": round(2.0 * M * N * K / ms / 1e9, 1)})
        del a, acc
    # the dX GEMM with the self-term backward (EPI 4): read g_z, x_dst [, g_prev], write C [, g_x_dst]
    for M, want_gx, with_prev in [(6_000_000, True, False), (3_000_000, True, True), (1_000_000, False, False)]:
        K = N = 256
        a = torch.randn(M, K, device="cuda")
        b = torch.randn(N, K, device="cuda") / K ** 0.5
        xd = torch.randn(M, N, device="cuda")
        eps = torch.tensor([0.3], device="cuda")
        prev = torch.randn(M, N, device="cuda") if with_prev else None
        ms = timeit(lambda: ops.gemm_nt_combine(a, b, xd, eps, 0, want_gx, g_prev=prev))
        byt = 4.0 * M * (K + N * (2 + (1 if want_gx else 0) + (1 if with_prev else 0)))
        out.append({"combine": True, "M": M, "want_gx": want_gx, "g_prev": with_prev, "ms": round(ms, 4),
                    "GB_s": round(byt / ms / 1e6, 1)})
        del a, xd, prev
    print(json.dumps({"HGIN_NT_WS32": os.environ.get("HGIN_NT_WS32", "1"), "shapes": out}))


if __name__ == "__main__":
    main()
