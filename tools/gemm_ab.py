"""Per-launch time of the fp32 GEMM shapes the cfg3 step runs, under the process-static HGIN_* switches of the
calling environment (one process per variant; tools/gpu_gemm_ab.sh runs the variants back to back).

    python tools/gemm_ab.py [--M 6000000] [--reps 10] [--only fwd512,fwd512acc,fwd256,dw512,dw256pro,dx256]

Prints one JSON line: {"env": {...}, "<shape>": {"ms": median ms per launch, "tflops_bf16_products": ...}, ...}.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gnn-link-prediction_amd")]

import torch  # noqa: E402

from hgin import _lib, ops  # noqa: E402


def timed(fn, reps):
    for _ in range(3):
        fn()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(reps + 1)]
    torch.cuda.synchronize()
    ev[0].record()
    for i in range(reps):
        fn()
        ev[i + 1].record()
    torch.cuda.synchronize()
    return statistics.median(ev[i].elapsed_time(ev[i + 1]) for i in range(reps))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=6_000_000)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--only", default="fwd512,fwd512acc,fwd256,dw512,dw256pro,dx256")
    ap.add_argument("--lib", default=None, help="A/B: load this libhgin.so instead of the in-tree build (same ABI)")
    ap.add_argument("--dtype", choices=("f32", "bf16"), default="f32",
                    help="bf16: the cfg5 kernels (operands and outputs bf16); GB_s = algorithmic bytes / time")
    args = ap.parse_args()
    if args.lib:
        _lib.build = lambda *a, **k: os.path.abspath(args.lib)   # (tools only: the product always builds its own)
    M = args.M
    bf = args.dtype == "bf16"
    sz = 2 if bf else 4
    g = torch.Generator(device="cuda").manual_seed(1)
    _randn = torch.randn

    def randn(*shape, **kw):   # operand tensors in the benchmarked dtype (scalars / bias stay fp32)
        t = _randn(*shape, **kw)
        return t.to(torch.bfloat16) if bf and len(shape) == 2 and shape[0] == M else t
    N = 256
    res = {"env": {k: v for k, v in os.environ.items() if k.startswith("HGIN_")}, "M": M, "lib": args.lib}
    s = torch.tensor([0.25], device="cuda")
    b = torch.randn(N, device="cuda", generator=g)
    for name in args.only.split(","):
        if name.startswith("fwd512two"):
            # the first layer's K = 512 forward as two K = 256 weight-stationary passes (a probe of its cost, not
            # the same arithmetic: pass 1 stores the fp32 product of the aggregate half, pass 2 takes it as its
            # accum row image — a real two-pass form would add it before the bias / PReLU, and carry the relation
            # sum's accum as a second row image)
            a = randn(M, 512, device="cuda", generator=g)
            w = (torch.randn(N, 512, device="cuda", generator=g) / 512 ** 0.5).to(a.dtype)
            w1, w2 = w[:, :256].contiguous(), w[:, 256:].contiguous()
            a1, a2 = a[:, :256].contiguous(), a[:, 256:].contiguous()
            byts = sz * (M * 512 + M * N * 2) + sz * 2 * M * N
            fn = lambda: ops.gin_mlp_fwd(a2, w2, b, s, ops.gemm_nt(a1, w1))   # noqa: E731
            flops = 2.0 * M * N * 512
        elif name == "fwdro":   # the readout's first Linear(512, 128) + PReLU forward ([x_path | raw] read in place; zy)
            a = randn(M, 512, device="cuda", generator=g)
            w = (torch.randn(128, 512, device="cuda", generator=g) / 512 ** 0.5).to(a.dtype)
            b128 = b[:128].contiguous()
            fn = lambda: ops.gin_mlp_fwd(a[:, :256], w, b128, s, None, comb2=a[:, 256:], zy=bf)   # noqa: E731
            byts = sz * M * (512 + 128 * (1 if bf else 2))    # (zy with a positive slope: y only)
            flops = 2.0 * M * 128 * 512
        elif name.startswith("fwd"):
            K = 512 if "512" in name else 256
            a = randn(M, K, device="cuda", generator=g)
            w = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).to(a.dtype)
            acc = randn(M, N, device="cuda", generator=g) if name.endswith("acc") else None
            byts = sz * (M * K + M * N * (2 + (acc is not None)))
            if K == 512:
                eps2 = torch.tensor([0.1], device="cuda")
                fn = lambda: ops.gin_mlp_fwd(a[:, :256], w, b, s, acc, comb2=a[:, 256:], eps2=eps2)   # noqa: E731
            else:
                fn = lambda: ops.gin_mlp_fwd(a, w, b, s, acc)   # noqa: E731
            flops = 2.0 * M * N * K
        elif name.startswith("dw"):
            K = 512 if "512" in name else 256
            a = randn(M, K, device="cuda", generator=g)
            gy = randn(M, N, device="cuda", generator=g)
            z = randn(M, N, device="cuda", generator=g)
            want = name.endswith("pro")
            byts = sz * M * (3 * N + K) if want else sz * M * (2 * N + K)
            if K == 512:
                fn = lambda: ops.mlp_bwd_w(gy, z, s, a[:, :256], a[:, 256:], want_gz=want)   # noqa: E731
            else:
                fn = lambda: ops.mlp_bwd_w(gy, z, s, a, want_gz=want)   # noqa: E731
            flops = 2.0 * M * N * K
        elif name == "dwro":   # the readout's first Linear(512, 128) dW with the PReLU backward (k_wsd_f32<128,512,PRO>)
            N = 128
            a = randn(M, 512, device="cuda", generator=g)
            gy = randn(M, N, device="cuda", generator=g)
            z = randn(M, N, device="cuda", generator=g)
            fn = lambda: ops.mlp_bwd_w(gy, z, s, a[:, :256], a[:, 256:], want_gz=True)   # noqa: E731
            byts = sz * M * (3 * N + 512)
            flops = 2.0 * M * N * 512
            N = 256
        elif name in ("dxro", "dx256p"):   # the plain dX GEMM at N = 256: the readout's (K = 128), the GIN width's
            K = 128 if name == "dxro" else 256
            gz = randn(M, K, device="cuda", generator=g)
            w = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).to(gz.dtype)
            byts = sz * M * (K + N)
            fn = lambda: ops.gemm_nt(gz, w)   # noqa: E731
            flops = 2.0 * M * N * K
        elif name == "dx256":
            gz = randn(M, N, device="cuda", generator=g)
            w = (torch.randn(N, N, device="cuda", generator=g) / 16).to(gz.dtype)
            xd = randn(M, N, device="cuda", generator=g)
            byts = sz * M * 4 * N
            eps = torch.tensor([0.1], device="cuda")
            fn = lambda: ops.gemm_nt_combine(gz, w.t().contiguous(), xd, eps, 0, want_gx=True)   # noqa: E731
            flops = 2.0 * M * N * N
        else:
            raise SystemExit(f"unknown shape {name}")
        with _lib.trace_launches() as tr:
            fn()
            torch.cuda.synchronize()
        ms = timed(fn, args.reps)
        res[name] = {"ms": round(ms, 4), "tflops_bf16_products": round((1 if bf else 6) * flops / (ms / 1e3) / 1e12, 1),
                     "GB_s": round(byts / (ms / 1e3) / 1e9, 1), "kernels": sorted(set(tr.kernels))}
        del fn
        torch.cuda.empty_cache()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
