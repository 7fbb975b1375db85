"""Probe: does a cfg3 aggregate (HBM-bound gather) overlap with a cfg3 fp32 GIN GEMM (MFMA / power-bound) when the
two run on separate streams, plain or CU-masked (hipExtStreamCreateWithCUMask)?  Prints one JSON line per case:
the wall time of the pair against the two run back to back.
    python tools/overlap_probe.py [--rows 3000000] [--reps 5]"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gnn-link-prediction_amd")]

import torch  # noqa: E402


def masked_stream(bits):
    """A torch stream over the CUs whose bits are set (256 bits: 8 words)."""
    hip = ctypes.CDLL("libamdhip64.so")
    words = (ctypes.c_uint32 * 8)()
    for b in bits:
        words[b // 32] |= 1 << (b % 32)
    h = ctypes.c_void_p()
    rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(h), 8, words)
    assert rc == 0, rc
    return torch.cuda.ExternalStream(h.value)


def main():
    from hgin import ops
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=3_000_000)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    dev = torch.device("cuda")
    torch.manual_seed(0)
    n_dst, n_src, E, F = args.rows, 2 * args.rows, 10 * args.rows, 256
    src = torch.randint(0, n_src, (E,), device=dev)
    dst = torch.randint(0, n_dst, (E,), device=dev)
    csr = ops.build_csr(torch.stack([src, dst]), 1, n_dst, n_src)
    del src, dst
    x = torch.randn(n_src, F, device=dev)
    agg = torch.empty(n_dst, F, device=dev)
    comb = torch.randn(n_dst, F, device=dev)
    w = torch.randn(F, F, device=dev) * 0.05
    b = torch.zeros(F, device=dev)
    a = torch.full((1,), 0.25, device=dev)

    def run_a():
        ops.aggregate_into(csr, x, None, None, ops.COMBINE_NONE, agg)

    def run_g():
        ops.gin_mlp_fwd(comb, w, b, a, None)

    def timed(fn):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ts = []
        for _ in range(args.reps + 1):
            torch.cuda.synchronize()
            s.record()
            fn()
            e.record()
            torch.cuda.synchronize()
            ts.append(s.elapsed_time(e))
        return sorted(ts[1:])[len(ts[1:]) // 2]

    def pair(sa, sg):
        def fn():
            cur = torch.cuda.current_stream()
            sa.wait_stream(cur)
            sg.wait_stream(cur)
            with torch.cuda.stream(sa):
                run_a()
            with torch.cuda.stream(sg):
                run_g()
            cur.wait_stream(sa)
            cur.wait_stream(sg)
        return fn

    ta, tg = timed(run_a), timed(run_g)
    tseq = timed(lambda: (run_a(), run_g()))
    out = {"agg_ms": round(ta, 3), "gemm_ms": round(tg, 3), "sequential_ms": round(tseq, 3)}
    out["plain_streams_ms"] = round(timed(pair(torch.cuda.Stream(), torch.cuda.Stream())), 3)
    s8 = masked_stream(range(0, 256, 32))   # 8 CUs: does the mask take effect at all?
    with torch.cuda.stream(s8):
        out["gemm_alone_on_8_ms"] = round(timed(run_g), 3)
    print(json.dumps(out), flush=True)
    for na in (32, 64, 96, 128):
        # every (256 / na)-th CU for the aggregate, spread over the XCDs; the rest for the GEMM
        step = 256 // na
        abits = [i for i in range(256) if i % step == 0]
        gbits = [i for i in range(256) if i % step != 0]
        sa, sg = masked_stream(abits), masked_stream(gbits)
        out[f"mask_{na}_{256 - na}_ms"] = round(timed(pair(sa, sg)), 3)
        with torch.cuda.stream(sa):
            out[f"agg_alone_on_{na}_ms"] = round(timed(run_a), 3)
        with torch.cuda.stream(sg):
            out[f"gemm_alone_on_{256 - na}_ms"] = round(timed(run_g), 3)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
