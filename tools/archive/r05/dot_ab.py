"""A/B of drhip_dot builds (DRHIP_DOT_BLOCKS_PER_CU variants, DRHIP_LIB per
child process): HIP-event time of the fused f32 dot at 2^27 and 2^29 pairs,
checked against torch fp64, interleaved rounds.
usage: python tools/archive/r05/dot_ab.py name=path ..."""
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
    for lg in (27, 29):
        n = 1 << lg
        x = torch.rand(n, device="cuda")
        y = torch.rand(n, device="cuda")
        p = torch.zeros(1, dtype=torch.float64, device="cuda")
        for _ in range(5):
            drhip.dot_async(0, np.float32, x.data_ptr(), y.data_ptr(), n, p.data_ptr())
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 100 if lg == 27 else 40
        e0.record(st)
        for _ in range(reps):
            drhip.dot_async(0, np.float32, x.data_ptr(), y.data_ptr(), n, p.data_ptr())
        e1.record(st)
        torch.cuda.synchronize()
        ref = float((x.double() * y.double()).sum().item())
        ms = e0.elapsed_time(e1) / reps
        out[lg] = {"ms": round(ms, 4), "frac": round(8.0 * n / (ms * 1e-3) / 8e12, 4), "rel": abs(float(p.item()) - ref) / ref}
print(json.dumps(out))
'''


def main():
    root = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))))
    variants = [a.split("=", 1) for a in sys.argv[1:]]
    for rep in range(3):
        for name, path in variants:
            env = dict(os.environ, ROOT=root, DRHIP_LIB=os.path.join(root, path))
            r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=300)
            line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
            print("rep", rep + 1, name, line[-1] if line else ("FAILED " + r.stderr[-500:]), flush=True)


if __name__ == "__main__":
    main()
