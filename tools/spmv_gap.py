"""Measurement tool (not product): the banded/random C4 SpMV kernel timed the
way bench.py times it (back-to-back launches, HIP events on the drhip stream)
and the way tools/spmv_sweep times it (a stream sync after every launch), on
buffers from torch's caching allocator and from drhip_malloc."""
import sys
import os
import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "distributed-ranges_amd"))
import drhip  # noqa: E402

drhip.init([0])
st = torch.cuda.ExternalStream(drhip.stream(0))
m = 1 << int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 26
reps = 10
for kind in (0, 1):
    nnz = drhip.csr_nnz(kind, 0, m, m, 10)
    byts = 8 * nnz + 4 * (m + 1) + 8 * m + 4 * m
    for alloc in ("torch", "drhip"):
        held = []
        if alloc == "torch":
            with torch.cuda.stream(st):
                rp = torch.empty(m + 1, dtype=torch.int32, device="cuda")
                ci = torch.empty(nnz, dtype=torch.int32, device="cuda")
                va = torch.empty(nnz, dtype=torch.float32, device="cuda")
                x = torch.rand(m, device="cuda")
                y = torch.zeros(m, device="cuda")
            P = [t.data_ptr() for t in (rp, ci, va, x, y)]
        else:
            P = [drhip.malloc(0, b) for b in (4 * (m + 1), 4 * nnz, 4 * nnz, 4 * m, 4 * m)]
            held = P
            drhip.fill(0, P[3], m, 0.5, np.float32)
            drhip.fill(0, P[4], m, 0.0, np.float32)
        drhip.csr_gen(0, kind, 0, m, m, 10, 1, P[0], P[1], P[2])
        torch.cuda.synchronize()
        for mode in ("back-to-back", "synced"):
            ev = []
            for r in range(reps + 2):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                drhip.spmv_csr(0, m, nnz, *P)
                e1.record(st)
                ev.append((e0, e1))
                if mode == "synced":
                    st.synchronize()
            torch.cuda.synchronize()
            ms = [a.elapsed_time(b) for a, b in ev[2:]]
            print(f"{'banded' if kind == 0 else 'random'} {alloc:5s} {mode:12s} mean {np.mean(ms):.4f} "
                  f"min {np.min(ms):.4f} ms  frac {byts / (np.mean(ms) * 1e-3) / 8e12:.3f}  "
                  f"addr%4096 {[p % 4096 for p in P]}", flush=True)
        for p in held:
            drhip.free(0, p)
        if alloc == "torch":
            del rp, ci, va, x, y
            torch.cuda.empty_cache()
drhip.finalize()
