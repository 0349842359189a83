"""Round 6 probe: drhip_sort of 2^28 4-byte keys under skewed digit
distributions (HIP-event ms per sort, median of 5 after a warm-up; checked
against torch.sort).  usage: python tools/r06/sort_skew_probe.py"""
import os
import sys

ROOT = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(ROOT, "distributed-ranges_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import drhip  # noqa: E402

drhip.init([0])
st = torch.cuda.ExternalStream(drhip.stream(0))
n = 1 << 28
g = torch.Generator(device="cuda").manual_seed(11)
with torch.cuda.stream(st):
    ws = drhip.sort_workspace(0, np.uint32, n)
    tmp = torch.empty(ws, dtype=torch.uint8, device="cuda")
    keys = torch.empty(n, dtype=torch.int32, device="cuda")


def case(name, npt, src):
    times = []
    for r in range(6):
        with torch.cuda.stream(st):
            keys.copy_(src.view(torch.int32))
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            drhip.sort_async(0, npt, keys.data_ptr(), n, tmp.data_ptr(), ws)
            e1.record(st)
        torch.cuda.synchronize()
        if r:
            times.append(e0.elapsed_time(e1))
    if npt == np.float32:
        ok = torch.equal(keys.view(torch.float32), torch.sort(src).values)
    else:
        ref = (torch.sort(src.to(torch.int64) & 0xFFFFFFFF).values).to(torch.int32)
        ok = torch.equal(keys, ref)
    print(f"{name:28s} {sorted(times)[2]:.3f} ms  ok {ok}", flush=True)


with torch.cuda.stream(st):
    u = torch.randint(-(1 << 31), (1 << 31) - 1, (n,), generator=g, device="cuda", dtype=torch.int32)
case("u32 uniform", np.uint32, u)
for bits in (24, 20, 16, 8):
    with torch.cuda.stream(st):
        s = torch.randint(0, 1 << bits, (n,), generator=g, device="cuda", dtype=torch.int32)
    case(f"u32 < 2^{bits}", np.uint32, s)
with torch.cuda.stream(st):
    c = torch.full((n,), 12345, device="cuda", dtype=torch.int32)
case("u32 constant", np.uint32, c)
with torch.cuda.stream(st):
    f = torch.randn(n, generator=g, device="cuda")
case("f32 randn", np.float32, f)
with torch.cuda.stream(st):
    f = torch.rand(n, generator=g, device="cuda")
case("f32 rand [0,1)", np.float32, f)
