"""A/B of reduce / scan builds on one box: each variant libdrhip.so
(DRHIP_LIB) in its own process, HIP-event timing of drhip_reduce and
drhip_inclusive_scan (f32 plus) at 2^27 and 2^30, interleaved rounds.
usage: python tools/reduce_ab.py name=path ...   (path "default" = the
in-tree build)"""
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
with torch.cuda.stream(st):
    for lg in (27, 30):
        n = 1 << lg
        x = torch.rand(n, device="cuda")
        p = torch.zeros(1, dtype=torch.float64, device="cuda")
        for _ in range(5):
            drhip.reduce_async(0, np.float32, "plus", x.data_ptr(), n, p.data_ptr())
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 100 if lg == 27 else 30
        e0.record(st)
        for _ in range(reps):
            drhip.reduce_async(0, np.float32, "plus", x.data_ptr(), n, p.data_ptr())
        e1.record(st)
        torch.cuda.synchronize()
        ref = float(x.double().sum().item())
        out[lg] = {"ms": e0.elapsed_time(e1) / reps, "rel": abs(float(p.item()) - ref) / ref}
        y = torch.empty_like(x)
        for _ in range(3):
            drhip.scan_async(0, np.float32, "plus", x.data_ptr(), y.data_ptr(), n)
        e0.record(st)
        for _ in range(reps):
            drhip.scan_async(0, np.float32, "plus", x.data_ptr(), y.data_ptr(), n)
        e1.record(st)
        torch.cuda.synchronize()
        out[lg]["scan_ms"] = e0.elapsed_time(e1) / reps
        out[lg]["scan_last_rel"] = abs(float(y[-1].item()) - ref) / ref
        del x, y
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
            r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=120)
            line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
            if r.returncode or not line:
                print(k, "FAILED", r.stderr[-800:], flush=True)
                return 1
            d = json.loads(line[-1])
            res[k].append(d)
            print(rnd, k, "reduce", {lg: round(v["ms"], 4) for lg, v in d.items()}, "scan",
                  {lg: round(v["scan_ms"], 4) for lg, v in d.items()}, {lg: v["rel"] for lg, v in d.items()},
                  flush=True)
    print(json.dumps(res))
    return 0


if __name__ == "__main__":
    sys.exit(main())
