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


def test_roofline_traffic_is_the_2p30_kernel():
    """roofline.traffic comes from the PMC summary profiles/pmc_current.json
    names, looked up by the exact instantiation the 2^30 step launches (a
    prefix match once returned the 2^27 small-tile kernel's bytes): the
    scan's bytes are within 1 % of 8 B x 2^30 and the reduce's of 4 B x 2^30."""
    sys.path.insert(0, ROOT)
    import json
    import bench
    cur = json.load(open(os.path.join(ROOT, "profiles", "pmc_current.json")))
    assert os.path.exists(os.path.join(ROOT, "profiles", cur["file"]))
    scan, src = bench.load_pmc("scan_wave_given_kernel<0, float, true, 32, 256>")
    red, _ = bench.load_pmc("reduce_tiles_kernel<0, float, 32>")
    assert src["file"] == "profiles/" + cur["file"] and src["commit"] == cur["commit"]
    assert abs(scan / (8 << 30) - 1) < 0.01 and abs(red / (4 << 30) - 1) < 0.01
    assert bench.load_pmc("scan_wave_given_kernel<0, float, true, 32, 256>", log2n=27)[0] is None
