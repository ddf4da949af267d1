"""bench.py's multi-GPU launcher (CPU, no GPU calls): `bench.py --gpus N` started without a
launcher starts N ranks itself from a parent that never touches the GPU, refuses a job larger
than the node, and passes its arguments through unchanged. Replaces the reference's
single-process nn.DataParallel (methods/_trainer.py:132, 167-168)."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_refuses_more_ranks_than_gpus():
    with pytest.raises(SystemExit, match="only 2 GPU"):
        bench.launch_ranks(8, ["--gpus", "8"], gpu_count=lambda: 2, run=lambda *a, **k: 0)


def test_launch_command_and_exit_status():
    seen = {}

    def run(cmd, env):
        seen["cmd"], seen["env"] = cmd, env
        return 3  # a failing rank's status comes back to the caller

    rc = bench.launch_ranks(4, ["--gpus", "4", "--steps", "7"], gpu_count=lambda: 8, run=run)
    assert rc == 3
    cmd = seen["cmd"]
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--nnodes=1" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert int(cmd[cmd.index("--master-port") + 1]) > 0
    assert cmd[-5:] == [os.path.abspath(bench.__file__), "--gpus", "4", "--steps", "7"]
    assert "WORLD_SIZE" not in seen["env"] or seen["env"]["WORLD_SIZE"] == os.environ.get("WORLD_SIZE")


def test_main_spawns_only_without_launcher(monkeypatch):
    calls = []
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(bench, "launch_ranks", lambda n, argv: calls.append((n, argv)) or 0)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2", "--steps", "3"])
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert e.value.code == 0 and calls == [(2, ["--gpus", "2", "--steps", "3"])]
    # --force-dist at N = 1 also goes through the launcher (a one-rank RCCL group)
    calls.clear()
    monkeypatch.setattr(sys, "argv", ["bench.py", "--force-dist"])
    with pytest.raises(SystemExit):
        bench.main()
    assert calls == [(1, ["--force-dist"])]


def test_rank_checks_world_against_gpus(monkeypatch):
    # a rank whose launcher started a different number of processes than --gpus asks for
    monkeypatch.setenv("WORLD_SIZE", "2")
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4"])
    with pytest.raises(SystemExit, match="WORLD_SIZE=2"):
        bench.main()
