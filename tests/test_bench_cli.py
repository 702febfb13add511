"""bench.py's launcher logic on the CPU (no device is touched).

``--gpus N`` without WORLD_SIZE re-launches itself under
torch.distributed.run with N processes on 127.0.0.1 and returns the child's
status; under a launcher, a WORLD_SIZE that disagrees with --gpus is an error.
"""
import sys

import pytest

import bench


def test_parse_defaults():
    a = bench.parse([])
    assert (a.gpus, a.scaling, a.dist_backend, a.rows) == (1, "strong", "nccl", 1_000_000)


def test_launch_builds_torchrun_command(monkeypatch):
    seen = {}

    def fake_call(cmd, env=None):
        seen["cmd"] = cmd
        return 7

    import subprocess

    monkeypatch.setattr(subprocess, "call", fake_call)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4", "--rows", "1000"])
    rc = bench.launch(bench.parse(["--gpus", "4", "--rows", "1000"]))
    assert rc == 7
    cmd = seen["cmd"]
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--master-addr=127.0.0.1" in cmd and "--nnodes=1" in cmd
    assert cmd[-4:] == ["--gpus", "4", "--rows", "1000"] and cmd[-5].endswith("bench.py")


def test_main_routes_to_launcher_without_world_size(monkeypatch):
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2"])
    monkeypatch.setattr(bench, "launch", lambda args: 3)
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert e.value.code == 3


def test_world_size_must_match_gpus(monkeypatch):
    monkeypatch.setenv("WORLD_SIZE", "2")
    with pytest.raises(SystemExit, match="WORLD_SIZE=2"):
        bench.Ranks(bench.parse(["--gpus", "3"]))
