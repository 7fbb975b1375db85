"""One side of an environment-switch A/B of the GEMM kernels: times the forward MLP GEMM (z, y, accum), the
dX NT GEMM and the dW TN GEMM at the given shapes and prints a bitwise digest of every output, so two runs
under different HGIN_* settings (separate processes: the switches are read once) can be compared line by
line (tools/ab_summary.py style).

    python tools/gemm_env_ab.py [--bf16] [--shapes=MxKxN,...] [--reps=N]
"""
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gnn-link-prediction_amd")]

import torch  # noqa: E402

from hgin import ops  # noqa: E402


def timeit(fn, reps):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def digest(*ts):
    h = hashlib.sha1()
    for t in ts:
        h.update(t.contiguous().view(torch.uint8).cpu().numpy().tobytes())
    return h.hexdigest()[:12]


def main():
    bf16 = "--bf16" in sys.argv
    dt = torch.bfloat16 if bf16 else torch.float32
    es = 2 if bf16 else 4
    reps = 10
    shapes = [(6_000_000, 512, 256), (3_000_000, 512, 256), (6_000_000, 256, 256)]
    for a in sys.argv[1:]:
        if a.startswith("--shapes="):
            shapes = [tuple(int(v) for v in s.split("x")) for s in a.split("=", 1)[1].split(",")]
        if a.startswith("--reps="):
            reps = int(a.split("=", 1)[1])
    for M, K, N in shapes:
        g = torch.Generator(device="cuda").manual_seed(0)
        a = torch.randn(M, K, device="cuda", generator=g).to(dt)
        w = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).to(dt)
        b = torch.randn(N, device="cuda", generator=g)
        s = torch.tensor([0.25], device="cuda")
        acc = torch.randn(M, N, device="cuda", generator=g).to(dt)
        gz = torch.randn(M, N, device="cuda", generator=g).to(dt)
        wt = w.t().contiguous()
        outs = {}
        cases = [
            ("mlp_fwd", lambda: outs.__setitem__("mlp_fwd", ops.gin_mlp_fwd(a, w, b, s, acc)),
             es * (M * K + 3 * M * N)),
            ("gemm_nt dX", lambda: outs.__setitem__("gemm_nt dX", (ops.gemm_nt(gz, wt),)), es * (M * N + M * K)),
            ("gemm_tn dW", lambda: outs.__setitem__("gemm_tn dW", (ops.gemm_tn(gz, a),)), es * (M * N + M * K)),
        ]
        res = {}
        for _ in range(3):
            for name, fn, _ in cases:
                res.setdefault(name, []).append(timeit(fn, reps))
        print(f"M={M} K={K} N={N} {dt}", flush=True)
        for name, _, byts in cases:
            t = sorted(res[name])[1]
            o = outs[name]
            o = [x for x in (o if isinstance(o, tuple) else (o,)) if isinstance(x, torch.Tensor)]
            print(f"   {name:12s} {t * 1e3:9.1f} us {byts / (t / 1e3) / 1e12:6.2f} TB/s "
                  f"{2.0 * M * N * K / (t / 1e3) / 1e12:7.1f} TF/s  digest {digest(*o)}", flush=True)
        del a, w, acc, gz, wt, outs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
