"""Measurement tool (not product): drhip_spmv_csr's CSR-stream shapes on the
C4 matrices (2^26 rows, banded and random), timed like bench.py
(back-to-back launches, HIP events on the drhip stream), interleaved over
rounds; every shape's y is compared bit for bit with the default's.
Shapes are env settings read by the launcher on every call:
DRHIP_SPMV_NPB_MAX (largest chunk), DRHIP_SPMV_NPB/_RPB (forced chunk),
DRHIP_SPMV_SPLIT (1: blocks own nonzero slots instead of row ranges)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "distributed-ranges_amd"))
import drhip  # noqa: E402

KEYS = ("DRHIP_SPMV_NPB", "DRHIP_SPMV_RPB", "DRHIP_SPMV_NPB_MAX", "DRHIP_SPMV_SPLIT")
SHAPES = [
    ("default", {}),
    ("row-blocks", {"DRHIP_SPMV_SPLIT": "0"}),
    ("nnz-split", {"DRHIP_SPMV_SPLIT": "1"}),
]
if len(sys.argv) > 1:
    SHAPES = [s for s in SHAPES if s[0] in sys.argv[1].split(",")]

drhip.init([0])
st = torch.cuda.ExternalStream(drhip.stream(0))
m = 1 << 26
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
    res = {name: [] for name, _ in SHAPES}
    same = {}
    for rnd in range(3):
        for name, env in SHAPES:
            for k in KEYS:
                os.environ.pop(k, None)
            os.environ.update(env)
            with torch.cuda.stream(st):
                y.zero_()
            drhip.spmv_csr(0, m, nnz, rp.data_ptr(), ci.data_ptr(), va.data_ptr(), x.data_ptr(), y.data_ptr())
            torch.cuda.synchronize()
            if ref is None:
                ref = y.clone()
            same[name] = bool(torch.equal(ref, y))
            ev = []
            for r in range(12):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                drhip.spmv_csr(0, m, nnz, rp.data_ptr(), ci.data_ptr(), va.data_ptr(), x.data_ptr(), y.data_ptr())
                e1.record(st)
                ev.append((e0, e1))
            torch.cuda.synchronize()
            res[name] += [a.elapsed_time(b) for a, b in ev[2:]]
    for name, _ in SHAPES:
        ms = np.array(res[name])
        print(f"{'banded' if kind == 0 else 'random'} {name:14s} mean {ms.mean():.4f} min {ms.min():.4f} ms "
              f"frac {byts / (ms.mean() * 1e-3) / 8e12:.3f} same_as_default {same[name]}", flush=True)
    del rp, ci, va, x, y, ref
    torch.cuda.empty_cache()
for k in KEYS:
    os.environ.pop(k, None)
drhip.finalize()
