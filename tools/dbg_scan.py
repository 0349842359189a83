"""Locate scan errors (measurement/debug tool): f32 plus-scan vs fp64 prefix."""
import sys
import numpy as np
sys.path.insert(0, "distributed-ranges_amd")
sys.path.insert(0, ".")
import drhip as dr
from oracle import oracle

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 25
dr.init([0])
x = np.random.default_rng(1).random(n, dtype=np.float32)
src = dr.DeviceArray(0, n, np.float32, host=x)
dst = dr.DeviceArray(0, n, np.float32)
dr.scan_async(0, np.float32, "plus", src.ptr, dst.ptr, n)
got = dst.numpy()
ref = np.cumsum(x.astype(np.float64))
rel = np.abs(got - ref) / np.maximum(ref, 1e-30)
bad = np.nonzero(rel > 1e-5)[0]
print("n", n, "max rel", rel.max(), "bad", bad.size)
if bad.size:
    T = 32768
    print("first bad", bad[:10], "tiles", np.unique(bad // T)[:20], "offsets in tile", np.unique(bad % T)[:20])
    i = bad[0]
    print("got", got[i - 2:i + 3], "ref", ref[i - 2:i + 3])
