"""Measurement tool (not product): drhip_spmv_csr's CSR-stream chunk shape
(DRHIP_SPMV_NPB nonzero slots, DRHIP_SPMV_RPB rows per block) on the C4
matrices, timed like bench.py (back-to-back launches, HIP events on the
drhip stream); every shape's y is compared bit for bit with the default's."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "distributed-ranges_amd"))
import drhip  # noqa: E402

drhip.init([0])
st = torch.cuda.ExternalStream(drhip.stream(0))
m = 1 << 26
SHAPES = [None, (2048, 204), (3072, 256), (1024, 102), (4096, 256), (2048, 128), (3072, 300 // 1)]
for kind in (0, 1):
    nnz = drhip.csr_nnz(kind, 0, m, m, 10)
    byts = 8 * nnz + 4 * (m + 1) + 8 * m + 4 * m
    with torch.cuda.stream(st):
        rp = torch.empty(m + 1, dtype=torch.int32, device="cuda")
        ci = torch.empty(nnz, dtype=torch.int32, device="cuda")
        va = torch.empty(nnz, dtype=torch.float32, device="cuda")
        x = torch.rand(m, device="cuda")
        y = torch.zeros(m, device="cuda")
    drhip.csr_gen(0, kind, 0, m, m, 10, 1, rp.data_ptr(), ci.data_ptr(), va.data_ptr())
    ref = None
    for rnd in range(2):
        for sh in SHAPES:
            if sh and sh[1] > 256:
                continue
            for k in ("DRHIP_SPMV_NPB", "DRHIP_SPMV_RPB"):
                os.environ.pop(k, None)
            if sh:
                os.environ["DRHIP_SPMV_NPB"], os.environ["DRHIP_SPMV_RPB"] = str(sh[0]), str(sh[1])
            with torch.cuda.stream(st):
                y.zero_()
            drhip.spmv_csr(0, m, nnz, rp.data_ptr(), ci.data_ptr(), va.data_ptr(), x.data_ptr(), y.data_ptr())
            torch.cuda.synchronize()
            if ref is None:
                ref = y.clone()
            same = bool(torch.equal(ref, y))
            ev = []
            for r in range(12):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                drhip.spmv_csr(0, m, nnz, rp.data_ptr(), ci.data_ptr(), va.data_ptr(), x.data_ptr(), y.data_ptr())
                e1.record(st)
                ev.append((e0, e1))
            torch.cuda.synchronize()
            ms = [a.elapsed_time(b) for a, b in ev[2:]]
            print(f"{'banded' if kind == 0 else 'random'} {str(sh or 'default'):12s} mean {np.mean(ms):.4f} "
                  f"min {np.min(ms):.4f} ms frac {byts / (np.mean(ms) * 1e-3) / 8e12:.3f} same_as_default {same}",
                  flush=True)
    del rp, ci, va, x, y, ref
    torch.cuda.empty_cache()
