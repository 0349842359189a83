"""Round 6 probe: does the dot kernel's time depend on where y sits relative
to x?  x and y (2^29 fp32 each) are carved from ONE allocation with y starting
2 GiB + off after x, for several offsets; plus the round-5 A/B layout (two
separate torch allocations) and the bench's layout.  Loop-timed (events
around back-to-back launches), three rounds.
usage: python tools/r06/dot_offsets.py"""
import json
import os
import sys

ROOT = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(ROOT, "distributed-ranges_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import drhip  # noqa: E402

drhip.init([0])
st = torch.cuda.ExternalStream(drhip.stream(0))
n = 1 << 29
reps = 40


def timed(xp, yp, p):
    for _ in range(5):
        drhip.dot_async(0, np.float32, xp, yp, n, p.data_ptr())
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(reps):
        drhip.dot_async(0, np.float32, xp, yp, n, p.data_ptr())
    e1.record(st)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


with torch.cuda.stream(st):
    p = torch.zeros(1, dtype=torch.float64, device="cuda")
    # offsets in elements after x's end (y = x + n + off)
    offs = [0, 1 << 10, 1 << 12, 1 << 14, 1 << 16, (1 << 18) + (1 << 10), 1 << 19, 3 << 17]
    big = torch.rand(2 * n + max(offs), device="cuda")
    sep_x = torch.rand(n, device="cuda")
    sep_y = torch.rand(n, device="cuda")
torch.cuda.synchronize()
print("separate allocations: x %#x y %#x (y - x = %d MiB)" % (sep_x.data_ptr(), sep_y.data_ptr(),
                                                             (sep_y.data_ptr() - sep_x.data_ptr()) >> 20))
for rnd in range(3):
    row = {}
    for off in offs:
        xp = big.data_ptr()
        yp = xp + 4 * (n + off)
        ms = timed(xp, yp, p)
        ref = float((big[:n].double() * big[n + off:2 * n + off].double()).sum().item()) if rnd == 0 else None
        if ref is not None:
            assert abs(p.item() - ref) <= 1e-5 * abs(ref), (p.item(), ref)
        row[f"y=x+2GiB+{4 * off >> 10}KiB"] = round(ms, 4)
    row["separate"] = round(timed(sep_x.data_ptr(), sep_y.data_ptr(), p), 4)
    row["same(x,x)"] = round(timed(big.data_ptr(), big.data_ptr(), p), 4)
    print("round", rnd + 1, json.dumps(row), flush=True)
