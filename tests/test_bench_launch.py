"""bench.py's multi-GPU entry without a launcher (CPU only, nothing is run):
`python bench.py --gpus N` with no WORLD_SIZE starts torch.distributed.run
as a child process with N ranks on 127.0.0.1 and returns its exit code,
before anything touches the GPU (no exec of the current process)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_self_launch_command(monkeypatch):
    sys.path.insert(0, ROOT)
    import bench
    seen = {}

    class R:
        returncode = 7

    def fake_run(cmd, *a, **kw):
        seen["cmd"] = cmd
        return R()

    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(subprocess, "run", fake_run)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4", "--steps", "3", "--warmup", "1"])
    assert bench.main() == 7
    cmd = seen["cmd"]
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--nnodes=1" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-7:] == [os.path.join(ROOT, "bench.py"), "--gpus", "4", "--steps", "3", "--warmup", "1"]
    assert "torch" not in sys.modules or not __import__("torch").cuda.is_initialized()
