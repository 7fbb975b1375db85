"""CPU-side static check of the weight-stationary bf16 GEMM kernels (k_ws_bf16): their counted-vmcnt DMA ring
is only correct when no instantiation spills to scratch or issues a compiler-visible VGPR-destination load in
its loop (tools/check_ws_asm.py compiles hgin_gemm_nt.hip to gfx950 assembly and inspects every instantiation)."""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc") and shutil.which("hipcc") is None,
                    reason="hipcc not available")
def test_ws_kernels_no_spill_no_loop_loads():
    p = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "check_ws_asm.py")], capture_output=True,
                       text=True, timeout=900)
    assert p.returncode == 0, p.stdout[-4000:] + p.stderr[-2000:]
    assert p.stdout.count("ok ") >= 40, p.stdout[-2000:]
