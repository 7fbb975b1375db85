"""The scaled two-term fp16 fp32 GEMM (HGIN_F32_GEMM=h2, hgin_gemm_nt.hip k_gemm_nt_h2) in a child interpreter
(the switch is process-static; tests/h2_child.py, started with subprocess, never an exec of this process)."""
import os
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.gpu
def test_h2_gemm_within_fp32_bound():
    env = {k: v for k, v in os.environ.items() if not k.startswith("HGIN_")}
    env["HGIN_F32_GEMM"] = "h2"
    p = subprocess.run([sys.executable, os.path.join(HERE, "h2_child.py")], env=env, capture_output=True, text=True,
                       timeout=300)
    assert p.returncode == 0, f"{p.stdout[-2000:]}\n{p.stderr[-4000:]}"
    assert "h2 child ok" in p.stdout
