"""One bf16 or fp32 weight-stationary dW shape, a few launches (a PMC target): the PReLU-fused form (g_z wanted,
k_wsd_*<N, K, PRO>) and the plain form on a materialised g_z (k_wsd_*<N, K>).
    python tools/wsd_one.py [bf16|f32] [pro|plain] M"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gnn-link-prediction_amd")]

import torch  # noqa: E402

from hgin import _lib, ops  # noqa: E402


def main():
    dt = torch.bfloat16 if sys.argv[1] == "bf16" else torch.float32
    pro = sys.argv[2] == "pro"
    M = int(sys.argv[3])
    g = torch.Generator(device="cuda").manual_seed(1)
    gy = torch.randn(M, 256, device="cuda", generator=g).to(dt)
    z = torch.randn(M, 256, device="cuda", generator=g).to(dt)
    b = torch.randn(M, 256, device="cuda", generator=g).to(dt)
    a = torch.tensor([0.25], device="cuda")
    fn = (lambda: ops.mlp_bwd_w(gy, z, a, b, want_gz=True)) if pro else (lambda: ops.gemm_tn(gy, b))  # noqa: E731
    with _lib.trace_launches() as tr:
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(5):
        fn()
    e.record()
    torch.cuda.synchronize()
    print(sys.argv[1:], f"{s.elapsed_time(e) / 5:.3f} ms", sorted(set(tr.kernels)), flush=True)


if __name__ == "__main__":
    main()
