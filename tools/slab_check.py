"""Bit-identity + timing of the weight-gradient slab reduction: one-launch k_slab_reduce vs the two-pass
k_slab_reduce1/2 (+ k_pro_final).  Run once per mode and compare the printed digests:

    HGIN_SLAB_REDUCE=2pass python tools/slab_check.py ; python tools/slab_check.py

Shapes: cfg2 / cfg5 dW shapes, a ragged N*K (not a multiple of 64 or 4), bf16 TN, and the fused
PReLU-backward dW (hgin_gin_mlp_bwd_w_f32: g_bias / g_prelu from the appended k_pro_final workgroups).
"""
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gnn-link-prediction_amd"))

import torch  # noqa: E402

from hgin import ops  # noqa: E402


def digest(*ts):
    h = hashlib.sha256()
    for t in ts:
        h.update(t.detach().float().cpu().contiguous().numpy().tobytes())
    return h.hexdigest()[:16]


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def main():
    mode = os.environ.get("HGIN_SLAB_REDUCE", "fused")
    dev = "cuda:0"
    g = torch.Generator(device=dev).manual_seed(0)
    cases = [("tn_f32_cfg2", 333334, 128, 256, torch.float32), ("tn_f32_ragged", 5003, 37, 91, torch.float32),
             ("tn_f32_small", 777, 8, 12, torch.float32), ("tn_bf16_cfg5", 1000000, 256, 512, torch.bfloat16)]
    for name, M, N, K, dt in cases:
        a = torch.randn(M, N, device=dev, generator=g).to(dt)
        b = torch.randn(M, K, device=dev, generator=g).to(dt)
        out = ops.gemm_tn(a, b)
        us = timed(lambda: ops.gemm_tn(a, b))
        ref = (a.double().T @ b.double())
        err = ((out.double() - ref).abs().max() / ref.abs().max()).item()
        print(f"{mode:6s} {name:14s} digest {digest(out)}  {us:8.1f} us/call  max rel err {err:.2e}", flush=True)
    for name, M, N, K in [("mlpw_cfg2", 333334, 128, 256), ("mlpw_ragged", 4099, 40, 72)]:
        g_y = torch.randn(M, N, device=dev, generator=g)
        z = torch.randn(M, N, device=dev, generator=g)
        b1 = torch.randn(M, K, device=dev, generator=g)
        slope = torch.full((1,), 0.25, device=dev)
        g_w, g_a, g_bias, _ = ops.mlp_bwd_w(g_y, z, slope, b1)
        us = timed(lambda: ops.mlp_bwd_w(g_y, z, slope, b1))
        print(f"{mode:6s} {name:14s} digest {digest(g_w, g_a, g_bias)}  {us:8.1f} us/call", flush=True)


if __name__ == "__main__":
    main()
