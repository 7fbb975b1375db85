"""bench.py's rank-launch decision (VERDICT r05 "next" 2): --gpus N > 1 must never produce an n_gpus: 1 line.

CPU only: the decision is taken before any HIP call, and these tests never reach one (dry runs, refused runs)."""
import json
import os
import subprocess
import sys

from conftest import ROOT

sys.path.insert(0, ROOT)
import bench  # noqa: E402

BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "HGIN_DIST_BACKEND")}
    env.update(kw)
    return env


def test_plan_single_gpu_runs_here():
    assert bench.launch_plan(1, {}, 0) == {"action": "run", "world": 1}
    assert bench.launch_plan(1, {"WORLD_SIZE": "1"}, 8) == {"action": "run", "world": 1}


def test_plan_multi_gpu_without_launcher_spawns_ranks():
    p = bench.launch_plan(8, {}, 8)
    assert p["action"] == "spawn" and p["world"] == 8
    argv = p["argv"]
    assert argv[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in argv and argv[argv.index("--master-addr") + 1] == "127.0.0.1"
    assert argv[-1] == os.path.abspath(BENCH)


def test_plan_refuses_what_it_cannot_honour():
    # too few devices on the node
    assert bench.launch_plan(8, {}, 4)["action"] == "error"
    # a launcher whose world size differs from --gpus
    assert bench.launch_plan(8, {"WORLD_SIZE": "1"}, 8)["action"] == "error"
    assert bench.launch_plan(2, {"WORLD_SIZE": "4"}, 8)["action"] == "error"
    assert bench.launch_plan(0, {}, 8)["action"] == "error"
    # the launcher's own ranks run
    assert bench.launch_plan(8, {"WORLD_SIZE": "8"}, 8) == {"action": "run", "world": 8}


def test_plan_gloo_rehearsal_shares_one_device():
    p = bench.launch_plan(2, {"HGIN_DIST_BACKEND": "gloo"}, 1)
    assert p["action"] == "spawn" and "--nproc-per-node=2" in p["argv"]


def test_dry_run_cli_touches_no_gpu():
    out = subprocess.run([sys.executable, BENCH, "--gpus", "8", "--launch-dry-run"], env=_env(), cwd=ROOT,
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    plan = json.loads(out.stdout.strip().splitlines()[-1])
    import torch
    want = "spawn" if torch.cuda.device_count() >= 8 else "error"
    assert plan["action"] == want


def test_mismatched_world_size_exits_nonzero_without_a_line():
    out = subprocess.run([sys.executable, BENCH, "--gpus", "8"], env=_env(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0"),
                         cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert out.returncode == 2
    assert "WORLD_SIZE=1" in out.stderr
    assert '"n_gpus"' not in out.stdout
