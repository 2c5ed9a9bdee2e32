"""bench.py's multi-rank launcher (CPU): `--gpus N` without a
torch.distributed environment starts N ranks through torch.distributed.run as
a child process (the parent never touches the GPU) and passes rank 0's line
through; a rank whose WORLD_SIZE disagrees with --gpus refuses to run."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_self_launch_command(monkeypatch):
    seen = {}

    def fake_call(cmd):
        seen["cmd"] = cmd
        return 7
    monkeypatch.setattr(subprocess, "call", fake_call)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4", "--steps", "3"])
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert e.value.code == 7  # the child's exit status
    cmd = seen["cmd"]
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert cmd[cmd.index("--nproc-per-node") + 1] == "4"
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert int(cmd[cmd.index("--master-port") + 1]) > 0
    assert cmd[-4:] == ["--gpus", "4", "--steps", "3"]
    assert cmd[-5].endswith("bench.py")


def test_world_size_must_match_gpus():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"],
                       env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 2
    assert "WORLD_SIZE=1 but --gpus 2" in r.stderr


def test_bad_gpu_count():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "0"],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "--gpus" in r.stderr
