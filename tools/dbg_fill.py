import sys, os, numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "distributed-ranges_amd"))
import drhip as dr
import ctypes as C
mode = sys.argv[1] if len(sys.argv) > 1 else "default"
dr.init([0])
tot = 0
for dtype in (np.int64, np.int32, np.float64):
    for n, off in ((4099, 0), (100003, 3), (100003, 0), (1 << 20, 1)):
        for rep in range(3):
            buf = dr.DeviceArray(0, n + off, dtype)
            dr.fill(0, buf.at(off), n, 7, dtype)
            dr.sync(0)
            if mode == "pinned":
                nb = (n + off) * np.dtype(dtype).itemsize
                hp = C.c_void_p(0)
                dr.check(dr.load().drhip_host_alloc(nb, C.byref(hp)))
                dr.check(dr.load().drhip_memcpy_d2h(0, hp, buf.ptr, nb))
                dr.sync(0)
                a = np.ctypeslib.as_array((C.c_char * nb).from_address(hp.value)).view(dtype).copy()[off:]
                dr.check(dr.load().drhip_host_free(hp))
            else:
                a = buf.numpy()[off:]
            bad = np.nonzero(a != 7)[0]
            tot += bad.size > 0
            buf.free()
print(mode, "failing cases:", tot, "of 36", flush=True)
dr.finalize()
