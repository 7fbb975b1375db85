"""Live per-kernel timing with HIP events recorded on the launching stream (torch's current stream, which
is the stream every libhgin.so call is enqueued on), plus the algorithmic work of each launch.

bench.py enables it over the timed region to report the aggregate kernel's achieved HBM bandwidth and the
MLP GEMM's achieved FLOP/s against the MI355X peaks (the numbers rocprofv3 --kernel-trace --stats
cross-checks in profiles/).
"""
from __future__ import annotations

from typing import Callable, Dict, List, Optional, Tuple

import torch

_probe: Optional["KernelProbe"] = None


class KernelProbe:
    def __init__(self):
        self.records: Dict[str, List[Tuple[torch.cuda.Event, torch.cuda.Event, float, float]]] = {}

    def around(self, kind: str, work: float, launch: Callable[[], None], nbytes: float = 0.0) -> None:
        """Time ``launch`` with events on the current stream; ``work`` is its algorithmic work (bytes for an
        HBM-bound kernel, FLOPs for a GEMM), ``nbytes`` a GEMM's algorithmic HBM bytes."""
        s = torch.cuda.Event(enable_timing=True)
        e = torch.cuda.Event(enable_timing=True)
        s.record()
        launch()
        e.record()
        self.records.setdefault(kind, []).append((s, e, float(work), float(nbytes)))

    def summary(self) -> Dict[str, dict]:
        torch.cuda.synchronize()
        out = {}
        for kind, recs in self.records.items():
            ms = sum(s.elapsed_time(e) for s, e, _, _ in recs)
            work = sum(w for _, _, w, _ in recs)
            nb = sum(b for _, _, _, b in recs)
            n = max(len(recs), 1)
            out[kind] = {"launches": len(recs), "total_ms": ms, "avg_ms": ms / n,
                         "work": work, "avg_work": work / n, "avg_bytes": nb / n,
                         "rate_per_s": work / (ms / 1e3) if ms > 0 else 0.0}
        return out


def start() -> KernelProbe:
    global _probe
    _probe = KernelProbe()
    return _probe


def stop() -> Optional[KernelProbe]:
    global _probe
    p, _probe = _probe, None
    return p


def active() -> Optional[KernelProbe]:
    return _probe


def gemm_bytes(M: int, N: int, K: int, s: int, z: bool, accum: bool) -> int:
    """Algorithmic HBM bytes of the forward MLP GEMM y = prelu(A W^T + b) [+ accum]: A read once, W once,
    y written, z written (saved for the backward) and accum read when present (s = element bytes)."""
    return s * (M * K + N * K + M * N * (1 + int(z) + int(accum)))


def aggregate_bytes(n_edges: int, n_rows: int, f_src: int, f_dst: int, mode: int, s: int = 4) -> int:
    """E*(I + s*F) + (N+1)*I + N*s*F_out  [+ N*s*F_dst read for the self term];
    s = 4 (fp32) or 2 (bf16)."""
    f_out = f_src + (f_dst if mode == 2 else 0)
    b = n_edges * (4 + s * f_src) + (n_rows + 1) * 4 + n_rows * s * f_out
    if mode != 0:
        b += n_rows * s * f_dst
    return b
