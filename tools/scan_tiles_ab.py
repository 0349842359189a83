"""A/B of the tile-prefix scan (drhip_reduce_tiles + drhip_inclusive_scan_tiles)
against the single-pass look-back scan, per libdrhip.so build (DRHIP_LIB),
each build in its own process, interleaved rounds; HIP-event timing per
kernel at 2^27 and 2^30 f32 plus.
usage: python tools/scan_tiles_ab.py name=path ...   ("default" = in-tree)"""
import json
import os
import subprocess
import sys

CHILD = r'''
import os, sys, json
sys.path.insert(0, os.path.join(os.environ["ROOT"], "distributed-ranges_amd"))
import numpy as np, torch, drhip
drhip.init([0])
st = torch.cuda.ExternalStream(drhip.stream(0))
out = {}


def timed(fn, reps):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(reps):
        fn()
    e1.record(st)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


with torch.cuda.stream(st):
    for lg in [int(v) for v in os.environ.get("LOG2S", "27,30").split(",")]:
        n = 1 << lg
        x = torch.rand(n, device="cuda")
        y = torch.empty_like(x)
        p = torch.zeros(1, dtype=torch.float64, device="cuda")
        reps = 100 if lg <= 27 else 20
        red = lambda: drhip.reduce_tiles_async(0, np.float32, "plus", x.data_ptr(), n, p.data_ptr())
        scn = lambda: drhip.scan_tiles_async(0, np.float32, "plus", x.data_ptr(), y.data_ptr(), n)
        one = lambda: drhip.scan_async(0, np.float32, "plus", x.data_ptr(), y.data_ptr(), n)
        red()
        scn()
        r = {"reduce_tiles_ms": timed(red, reps), "scan_tiles_ms": timed(scn, reps)}
        torch.cuda.synchronize()
        ref = torch.cumsum(x.double(), 0)
        r["tiles_rel"] = float(((y.double() - ref).abs() / ref).max().item())
        one()
        r["single_pass_ms"] = timed(one, reps)
        r["single_rel"] = float(((y.double() - ref).abs() / ref).max().item())
        out[lg] = r
        del x, y, ref
        torch.cuda.empty_cache()
print(json.dumps(out))
drhip.finalize()
'''


def main():
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    vs = [a.split("=", 1) for a in sys.argv[1:]]
    res = {k: [] for k, _ in vs}
    for rnd in range(3):
        for k, path in vs:
            env = dict(os.environ, ROOT=root)
            if path != "default":
                env["DRHIP_LIB"] = os.path.abspath(path)
            r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=150)
            line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
            if r.returncode or not line:
                print(k, "FAILED", r.stderr[-800:], flush=True)
                return 1
            d = json.loads(line[-1])
            res[k].append(d)
            print(rnd, k, {lg: {kk: round(vv, 4) if kk.endswith("ms") else vv for kk, vv in v.items()}
                           for lg, v in d.items()}, flush=True)
    print(json.dumps(res))
    return 0


if __name__ == "__main__":
    sys.exit(main())
