"""Stress check: fused dW GEMM with the g_z output (hgin_gin_mlp_bwd_w_f32) followed by the dX GEMM on g_z,
repeated; reports which stage first disagrees with a torch reference."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gnn-link-prediction_amd")]
import torch  # noqa: E402

from hgin import ops  # noqa: E402

torch.manual_seed(0)
M, N, K1, K2 = 3000, 128, 128, 128
for it in range(int(sys.argv[1]) if len(sys.argv) > 1 else 50):
    gy = torch.randn(M, N, device="cuda")
    z = torch.randn(M, N, device="cuda")
    a = torch.tensor([0.25], device="cuda")
    x1 = torch.randn(M, K1, device="cuda")
    x2 = torch.randn(M, K2, device="cuda")
    W = torch.randn(N, K1 + K2, device="cuda") / 16
    g_w, g_a, g_b, g_z = ops.mlp_bwd_w(gy, z, a, x1, x2, want_gz=True)
    gx1 = ops.gemm_nt(g_z, W[:, :K1].t().contiguous())
    torch.cuda.synchronize()
    ref = torch.where(z > 0, gy, a * gy)
    bad = (g_z != ref).any(1).nonzero().flatten()
    rx = ref.double() @ W[:, :K1].double()
    ex = (gx1.double() - rx).abs().max().item()
    rw = ref.double().t() @ torch.cat((x1, x2), 1).double()
    ew = ((g_w.double() - rw).norm() / rw.norm()).item()
    if bad.numel() or ex > 1e-3 or ew > 1e-5:
        print(f"iter {it}: g_z bad rows {bad[:10].tolist()} ({bad.numel()}), dX max err {ex:.3g}, dW rel {ew:.3g}")
    else:
        print(f"iter {it}: ok (dX {ex:.2g}, dW {ew:.2g})")
