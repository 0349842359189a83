"""Round 6 probe: drhip_sort per key type at 1 GiB of keys (2^28 4-byte or
2^27 8-byte keys), HIP-event ms per sort (median of 5 after a warm-up),
checked against torch.sort.  usage: python tools/r06/sort64_probe.py"""
import os
import sys

ROOT = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(ROOT, "distributed-ranges_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import drhip  # noqa: E402

drhip.init([0])
st = torch.cuda.ExternalStream(drhip.stream(0))
cases = [("u32", np.uint32, torch.int32, 28), ("f32", np.float32, torch.float32, 28),
         ("u64", np.uint64, torch.int64, 27), ("f64", np.float64, torch.float64, 27)]
for name, npt, tt, lg in cases:
    n = 1 << lg
    with torch.cuda.stream(st):
        g = torch.Generator(device="cuda").manual_seed(7)
        if tt.is_floating_point:
            src = torch.randn(n, generator=g, device="cuda", dtype=tt)
        else:
            src = torch.randint(-(1 << 62) if tt == torch.int64 else -(1 << 31), (1 << 62) if tt == torch.int64 else (1 << 31) - 1,
                                (n,), generator=g, device="cuda", dtype=tt)
        keys = torch.empty_like(src)
        ws = drhip.sort_workspace(0, npt, n)
        tmp = torch.empty(ws, dtype=torch.uint8, device="cuda")
    times = []
    for r in range(6):
        with torch.cuda.stream(st):
            keys.copy_(src)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            drhip.sort_async(0, npt, keys.data_ptr(), n, tmp.data_ptr(), ws)
            e1.record(st)
        torch.cuda.synchronize()
        if r:
            times.append(e0.elapsed_time(e1))
    # unsigned order for the unsigned types: compare through the same bit view torch sorts
    if name == "u32":
        ref = torch.sort(src.view(torch.int32).to(torch.int64) & 0xFFFFFFFF).values.to(torch.int32)
        ok = torch.equal(keys.view(torch.int32), ref.view(torch.int32))
    elif name == "u64":
        flip = src ^ torch.tensor(-(1 << 63), dtype=torch.int64, device="cuda")  # unsigned order as signed
        ref = torch.sort(flip).values ^ torch.tensor(-(1 << 63), dtype=torch.int64, device="cuda")
        ok = torch.equal(keys, ref)
    else:
        ok = torch.equal(keys, torch.sort(src).values)
    ms = sorted(times)[len(times) // 2]
    passes = 4 if lg == 28 else 8
    print(f"{name}: 2^{lg} keys ({passes} passes) {ms:.3f} ms  {n / ms / 1e6:.1f} Gkeys/s  "
          f"{(4 if lg == 28 else 8) * n * (1 + 2 * passes) / 8 * 8 / (ms * 1e-3) / 1e12:.2f} TB/s model  ok {ok}", flush=True)
    del src, keys, tmp
    torch.cuda.empty_cache()
