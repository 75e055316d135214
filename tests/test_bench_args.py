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


def test_exchange_model_arithmetic():
    """bench.py's `exchange.model` (tools/step_model.exchange_model): the
    measured receive / per-link rate from the exchange-only time, and the
    step the model predicts at that rate beside the measured step."""
    import step_model as M
    # W = 2, fp32 n = 10M: 20 MB into each rank; exchange alone 0.5 ms → 40 GB/s over one link
    r = M.exchange_model(2, 1, False, 10_000_000, 4, 0.2, 0.3, 0.5, 0.9)
    assert r["bytes_in_per_step"] == 20e6
    assert abs(r["recv_GBps"] - 40.0) < 1e-9 and abs(r["link_GBps"] - 40.0) < 1e-9
    # K = 1 plain: stage + reduce, then the whole exchange, serial → 0.2 + 0.1 + 0.5
    assert abs(r["predicted_step_ms"] - 0.8) < 1e-9
    assert abs(r["measured_over_predicted"] - 0.9 / 0.8) < 1e-9
    # at 50 GB/s per link the exchange takes 0.4 ms
    r = M.exchange_model(2, 1, False, 10_000_000, 4, 0.2, 0.3, 0.5, 0.9, assumed_link_GBps=(50.0,))
    assert abs(r["at_assumed_link_rates"][0]["step_ms"] - 0.7) < 1e-9
    # W = 8: 7/8 of y arrives over 7 links; K = 4 chained overlaps the exchange with the next stage
    r = M.exchange_model(8, 4, True, 10_000_000, 8, 0.05, 0.15, 0.2, 0.2)
    assert abs(r["bytes_in_per_step"] - 70e6) < 1e-3
    assert abs(r["link_GBps"] - 70e6 / 0.2e-3 / 1e9 / 7) < 1e-9
    assert r["mode"] == "chained" and 0.15 <= r["predicted_step_ms"] <= 0.05 + 0.15 + 0.2
    assert abs(r["predicted_step_ms"] - M.simulate(0.05, 0.10, 0.2, 4, True)) < 1e-12
    # one rank: no exchange, no rate
    assert "link_GBps" not in M.exchange_model(1, 1, False, 100, 4, 0.1, 0.2, 0.0, 0.2)
