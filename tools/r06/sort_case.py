"""Round 6 probe: drhip_sort of ONE key distribution, 2^28 keys, 6 sorts
(for rocprofv3 kernel stats).  usage: python tools/r06/sort_case.py u32|f32rand|f32randn|u16"""
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
kind = sys.argv[1]
g = torch.Generator(device="cuda").manual_seed(5)
with torch.cuda.stream(st):
    if kind == "u32":
        src, npt = torch.randint(-(1 << 31), (1 << 31) - 1, (n,), generator=g, device="cuda", dtype=torch.int32), np.uint32
    elif kind == "u16":
        src, npt = torch.randint(0, 1 << 16, (n,), generator=g, device="cuda", dtype=torch.int32), np.uint32
    elif kind == "f32rand":
        src, npt = torch.rand(n, generator=g, device="cuda"), np.float32
    else:
        src, npt = torch.randn(n, generator=g, device="cuda"), np.float32
    keys = torch.empty_like(src)
    ws = drhip.sort_workspace(0, npt, n)
    tmp = torch.empty(ws, dtype=torch.uint8, device="cuda")
    for _ in range(6):
        keys.copy_(src)
        drhip.sort_async(0, npt, keys.data_ptr(), n, tmp.data_ptr(), ws)
torch.cuda.synchronize()
print(kind, "done")
