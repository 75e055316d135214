"""bench.py --gpus N argument handling: N > 1 without
a launcher starts N ranks itself (torch.distributed.run as a child process),
a mismatch with the launcher's WORLD_SIZE or with the visible GPUs refuses to
run.  CPU only: launch_decision() is pure, and the refusal path exits before
any GPU call."""
import os
import subprocess
import sys

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_single_gpu_runs_in_process():
    assert bench.launch_decision(1, {}, 1, ["--steps", "3"]) == ("run", None)
    assert bench.launch_decision(1, {}, 0, []) == ("run", None)


def test_under_launcher_matching_world_runs():
    env = {"WORLD_SIZE": "8", "RANK": "3", "LOCAL_RANK": "3"}
    assert bench.launch_decision(8, env, 8, []) == ("run", None)
    # the world-1 native rehearsal (LHPC_DIST_NATIVE=1, one launcher rank)
    assert bench.launch_decision(1, {"WORLD_SIZE": "1"}, 1, []) == ("run", None)


def test_under_launcher_mismatch_refuses():
    for gpus, ws in ((8, "1"), (2, "4"), (1, "2")):
        action, msg = bench.launch_decision(gpus, {"WORLD_SIZE": ws}, 8, [])
        assert action == "refuse" and f"WORLD_SIZE={ws}" in msg


def test_no_launcher_spawns_n_ranks_with_same_args():
    argv = ["--gpus", "8", "--steps", "20", "--warmup", "5", "--workload", "c3"]
    action, cmd = bench.launch_decision(8, {}, 8, argv, port=29611)
    assert action == "spawn"
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd
    assert "--master-addr=127.0.0.1" in cmd and "--master-port=29611" in cmd
    i = cmd.index(os.path.join(bench.ROOT, "bench.py"))
    assert cmd[i + 1:] == argv  # the ranks run exactly the caller's arguments


def test_more_ranks_than_gpus_refuses_unless_gloo():
    action, msg = bench.launch_decision(2, {}, 1, ["--gpus", "2"])
    assert action == "refuse" and "1 GPU(s) visible" in msg
    action, cmd = bench.launch_decision(2, {"LHPC_DIST_BACKEND": "gloo"}, 1, ["--gpus", "2"])
    assert action == "spawn" and "--nproc-per-node=2" in cmd
    action, _ = bench.launch_decision(4, {"LHPC_DIST_BACKEND": "nccl"}, 2, [])
    assert action == "refuse"


def test_refusal_exits_nonzero_before_any_gpu_call():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK",
                                                              "LHPC_DIST_BACKEND")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert "GPU(s) visible" in r.stderr and not r.stdout.strip()


def test_spmv_options_forms():
    assert bench.parse_options(None) is None
    assert bench.parse_options('{"xtile_steps": 4}') == {"xtile_steps": 4}
    assert bench.parse_options("xtile_steps=4,xtile_piece=150000") == {"xtile_steps": 4, "xtile_piece": 150000}
