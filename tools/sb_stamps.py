"""Diagnostic: where the fused small-batch step's readout and weight-gradient launches spend their time.
    python tools/sb_stamps.py --build        # here: libhgin.so with -DHGIN_SB_STAMPS into hgin/_build_diag/
    python tools/sb_stamps.py                # on the GPU: runs the step, prints the last step's phase shares
The stamps (wall clock, 100 MHz) come from thread 0 of each workgroup at its phase boundaries (csrc/hgin_smallbatch.hip
SB_STAMP); the diagnostic build's run time is not quoted anywhere, only its phase shares."""
import argparse
import ctypes
import glob
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "gnn-link-prediction_amd")
sys.path[:0] = [ROOT, PKG]
DIAG = os.path.join(PKG, "hgin", "_build_diag")
# stamp index -> the phase it closes (csrc/hgin_smallbatch.hip SB_STAMP; nhid <= 2: the backward of layer i closes
# at 8 + 2 i (g_z) and 9 + 2 i (g_in), the slope sum at 12, the gpath store at 13)
RO_PHASES = {1: "stage", 2: "in0", 3: "fwd0", 4: "fwd1", 5: "fwd2", 6: "head", 7: "gseed", 8: "gz0", 9: "gin0",
             10: "gz1", 11: "gin1", 12: "slope", 13: "gpath"}


def build():
    from hgin import _lib
    _lib.build()
    os.makedirs(DIAG, exist_ok=True)
    src = os.path.join(_lib.CSRC, "hgin_smallbatch.hip")
    obj = os.path.join(DIAG, "hgin_smallbatch.o")
    flags = [f for f in _lib.HIPCC_FLAGS if f != "-shared"]
    subprocess.run([_lib._hipcc()] + flags + ["-DHGIN_SB_STAMPS", "-I", _lib.INCLUDE, "-c", "-o", obj, src], check=True)
    objs = [o for o in sorted(glob.glob(os.path.join(_lib.BUILD_DIR, "*.o"))) if not o.endswith("hgin_smallbatch.o")]
    subprocess.run([_lib._hipcc(), "-shared", "-fPIC", f"--offload-arch={_lib.ARCH}", "-o",
                    os.path.join(DIAG, "libhgin.so"), obj] + objs, check=True)
    print("built", os.path.join(DIAG, "libhgin.so"))


def run(steps):
    import numpy as np
    import torch
    from hgin import _lib
    _lib.build = lambda *a, **k: os.path.join(DIAG, "libhgin.so")
    from hgin import HetroGIN
    from hgin.data import CONFIGS, scaled_config, synthetic_graph
    from hgin.smallbatch import SmallBatchStep
    from hgin.store import GraphStore
    dev = torch.device("cuda")
    base = CONFIGS["cfg1"]
    rng = np.random.default_rng(0)
    graphs = [synthetic_graph(scaled_config(base, float(rng.uniform(0.5, 1.5)), name=f"g{i}"), seed=i)
              for i in range(256)]
    store = GraphStore.build(graphs, device=dev, normalize=True)
    order = [rng.choice(256, 8, replace=False).tolist() for _ in range(5 + steps)]
    torch.manual_seed(1997)
    model = HetroGIN(**base.model_kwargs({"link": base.f_link, "path": base.f_path, "node": base.f_node})).to(dev)
    opt = torch.optim.Adam(lr=1e-3, params=model.parameters())
    st = SmallBatchStep(model, opt, store, 8, warmup_ids=order[:5], warmup=5)
    lib = _lib.lib()
    n = 1024 * 16 + 2 * 2048 * 2
    buf = (ctypes.c_ulonglong * n)()
    fn = lib.hgin_sb_stamps_read
    fn.argtypes, fn.restype = [ctypes.c_void_p, ctypes.c_int64], ctypes.c_int
    shares = []
    for ids in order[5:]:
        torch.cuda.synchronize()
        ctypes.memset(buf, 0, ctypes.sizeof(buf))
        st.step(ids)
        torch.cuda.synchronize()
        assert fn(buf, n) == 0
        a = np.frombuffer(buf, dtype=np.uint64).astype(np.int64)
        ro = a[:1024 * 16].reshape(1024, 16)
        act = ro[:, 0] > 0
        ro = ro[act]
        t0 = ro[:, 0].min()
        ro = np.where(ro > 0, ro - t0 + 1, 0)   # (unwritten stamps stay 0)
        w = a[1024 * 16:].reshape(2, 2048, 2)
        shares.append((ro, w, t0, int(act.sum())))
    ro, w, t0, nact = shares[-1]
    print(f"readout: {nact} active workgroups; times in us from the first workgroup's start (10 ns ticks)")
    print(f"  start: min 0  median {np.median(ro[:, 0]) / 100:.2f}  max {ro[:, 0].max() / 100:.2f}")
    print(f"  end:   median {np.median(ro[:, 13]) / 100:.2f}  max {ro[:, 13].max() / 100:.2f}")
    prev = ro[:, 0]
    cols = [k for k in RO_PHASES if (ro[:, k] > 0).all()]
    for k in sorted(cols, key=lambda k: np.median(ro[:, k])):   # in time order
        col = ro[:, k]
        d = (col - prev) / 100.0
        print(f"  {RO_PHASES[k]:6s} median {np.median(d):6.2f} us  p90 {np.percentile(d, 90):6.2f}  max {d.max():6.2f}")
        prev = col
    for l in (1, 0):
        ww = w[l]
        ok = ww[:, 0] > 0
        s, e = ww[ok, 0], ww[ok, 1]
        d = (e - s) / 100.0
        base_t = s.min()
        print(f"bwd_w (layer parity {l}): {ok.sum()} blocks; start spread {(s.max() - base_t) / 100:.2f} us, "
              f"end {(e.max() - base_t) / 100:.2f} us; block time median {np.median(d):.2f} p90 "
              f"{np.percentile(d, 90):.2f} max {d.max():.2f} us")
        idx = np.nonzero(ok)[0]
        # blocks y-major: block id = y * 128 + x (n_parts = 128)
        ys = idx // 128
        for y in sorted(set(ys.tolist())):
            dd = d[ys == y]
            print(f"    y={y}: median {np.median(dd):.2f} max {dd.max():.2f} us")


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--steps", type=int, default=20)
    args = ap.parse_args()
    build() if args.build else run(args.steps)
