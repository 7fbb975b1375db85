"""Digest of the PReLU / combine backward outputs (g_z, g_prelu, g_bias; g_x, g_eps) at cfg2 / cfg5 / ragged
shapes: run once per row-kernel variant (HGIN_ROWS_*) and compare, the variants must be bit-identical."""
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gnn-link-prediction_amd")]

import torch  # noqa: E402

from hgin import ops  # noqa: E402

h = hashlib.sha256()
g = torch.Generator(device="cuda").manual_seed(0)
a = torch.tensor([0.25], device="cuda")
for dt in (torch.float32, torch.bfloat16):
    for M, N in ((333334, 128), (3000000, 256), (1001, 36)):
        gy = torch.randn(M, N, device="cuda", generator=g).to(dt)
        z = torch.randn(M, N, device="cuda", generator=g).to(dt)
        for t in ops.prelu_bwd(gy, z, a):
            h.update(t.float().cpu().numpy().tobytes())
        for t in ops.combine_bwd(gy, z, a, True):
            h.update(t.float().cpu().numpy().tobytes())
print("rows digest", {k: v for k, v in os.environ.items() if k.startswith("HGIN_ROWS")}, h.hexdigest()[:16])
