"""Static check of the weight-stationary kernels (k_ws_bf16 / k_ws_f32 / k_wss_f32 in hgin_gemm_nt.hip, k_wsd_* / k_wsp_f32 / k_wsp_bf16
in hgin_gemm_tn.hip)
in their gfx950 assembly: the
counted-vmcnt ring is only correct when the loop holds no compiler-visible vector-memory load (the compiler's
own waits would not count the inline-asm DMAs), so every instantiation must have no scratch (spill) traffic,
and its only global loads must be the W-slice / bias loads of the prologue.

    python tools/check_ws_asm.py            # compiles to a temporary .s and prints one line per kernel
"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRCS = [os.path.join(ROOT, "gnn-link-prediction_amd", "csrc", f) for f in ("hgin_gemm_nt.hip", "hgin_gemm_tn.hip")]


def main():
    s = ""
    with tempfile.TemporaryDirectory() as d:
        for i, src in enumerate(SRCS):
            out = os.path.join(d, f"k{i}.s")
            cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-ffp-contract=off", "--offload-arch=gfx950",
                   "--offload-device-only", "-S", "-I", os.path.join(ROOT, "include"), "-o", out, src]
            subprocess.run(cmd, check=True, capture_output=True)
            s += open(out).read()
    bad = 0
    for m in re.finditer(r"^(_ZN4hgin12_GLOBAL__N_1\d+k_ws(?:[dp]?_bf16|[dps]?_f32)\S*):", s, re.M):
        body = s[m.end():s.index(".Lfunc_end", m.end())]
        loop = body[body.find("Loop Header"):] if "Loop Header" in body else body
        scratch = len(re.findall(r"\bscratch_(load|store)|buffer_(load|store)_dword\S* \S+, off, s\[0:3\]", body))
        loads_in_loop = len(re.findall(r"\bglobal_load_(?!lds)\w+", loop))
        waits = sorted(set(int(x) for x in re.findall(r"s_waitcnt vmcnt\((\d+)\)", loop)))
        nm = re.search(r"(k_ws(?:[dp]?_bf16|[dps]?_f32)(?:I.*?EEEv|(?=P)))", m.group(1))
        name = nm.group(1) if nm else m.group(1)
        ok = scratch == 0 and loads_in_loop == 0
        bad += not ok
        print(f"{'ok ' if ok else 'BAD'} {name}: scratch ops {scratch}, VGPR-destination global loads in the loop "
              f"{loads_in_loop}, loop vmcnt waits {waits}")
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
