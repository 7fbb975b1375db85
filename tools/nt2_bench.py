"""LDS-DMA NT GEMM (k_nt2, B pre-converted by hgin_nt_planes_*) vs the register-staged k_gemm_nt on the cfg3 /
cfg5 shapes: bitwise comparison of z / y, and interleaved timing rounds (median).

    python tools/nt2_bench.py [--bf16] [--shapes=MxKxN,...]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gnn-link-prediction_amd")]

os.environ["HGIN_NT2"] = "1"   # before libhgin / hgin.ops read it
import torch  # noqa: E402

from hgin import _lib, ops  # noqa: E402
from hgin.ops import _p, _stream  # noqa: E402


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
    bf16 = "--bf16" in sys.argv
    dt = torch.bfloat16 if bf16 else torch.float32
    sfx = "bf16" if bf16 else "f32"
    es = 2 if bf16 else 4
    shapes = [(6_000_000, 512, 256), (6_000_000, 256, 256), (3_000_000, 512, 256), (1_000_000, 512, 256),
              (6_000_000, 512, 128), (6_000_000, 256, 512)]
    for a in sys.argv[1:]:
        if a.startswith("--shapes="):
            shapes = [tuple(int(v) for v in s.split("x")) for s in a.split("=", 1)[1].split(",")]
    for M, K, N in shapes:
        g = torch.Generator(device="cuda").manual_seed(0)
        a = torch.randn(M, K, device="cuda", generator=g).to(dt)
        w = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).to(dt)
        b = torch.randn(N, device="cuda", generator=g)
        s = torch.tensor([0.25], device="cuda")
        acc = torch.randn(M, N, device="cuda", generator=g).to(dt)
        outs = {}
        planes = ops.nt_planes(w)
        assert planes is not None
        for name, pl in (("old", None), ("nt2", planes)):
            z = torch.empty(M, N, device="cuda", dtype=dt)
            y = torch.empty(M, N, device="cuda", dtype=dt)

            def run(z=z, y=y, pl=pl):
                _lib.call(f"hgin_gin_mlp_fwd_{sfx}", _p(a), a.stride(0), K, None, 0, None, _p(w), _p(b), _p(s),
                          _p(acc), _p(z), _p(y), M, N, K, _p(pl), _stream(a))
            outs[name] = (run, z, y)
        outs["old"][0]()
        outs["nt2"][0]()
        torch.cuda.synchronize()
        same_z = torch.equal(outs["old"][1], outs["nt2"][1])
        same_y = torch.equal(outs["old"][2], outs["nt2"][2])
        ts = {"old": [], "nt2": []}
        for _ in range(3):
            for name in ("old", "nt2"):
                ts[name].append(timeit(outs[name][0]))
        nbytes = es * (M * K + N * K + 3 * M * N)
        flops = 2.0 * M * N * K
        line = f"{sfx} M={M} K={K} N={N}: bitwise z {same_z} y {same_y}"
        for name in ("old", "nt2"):
            t = sorted(ts[name])[1]
            line += (f" | {name} {t * 1e3:8.1f} us {nbytes / (t / 1e3) / 1e12:5.2f} TB/s "
                     f"{flops / (t / 1e3) / 1e12:6.1f} TF/s")
        print(line, flush=True)
        del a, w, acc, outs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
