"""GPU parity for the elementwise family (fill / iota / for_each forms),
the 1-D/2-D stencil kernels with halo exchange, and the CSR SpMV."""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "shp_known_answers.json")


@pytest.mark.parametrize("dtype", [np.int32, np.float32, np.int64, np.float64, np.uint32])
@pytest.mark.parametrize("n,off", [(1, 0), (10, 1), (4099, 0), (100003, 3)])
def test_fill_iota_transform(dr, dtype, n, off):
    buf = dr.DeviceArray(0, n + off, dtype)
    dr.fill(0, buf.at(off), n, 7, dtype)
    assert np.all(buf.numpy()[off:] == 7)
    dr.iota(0, buf.at(off), n, 20, dtype)
    assert np.array_equal(buf.numpy()[off:], (np.arange(n) + 20).astype(dtype))
    dr.transform_scalar(0, dtype, "mul", buf.at(off), buf.at(off), n, 3)
    assert np.array_equal(buf.numpy()[off:], ((np.arange(n) + 20) * 3).astype(dtype))
    other = dr.DeviceArray(0, n + off, dtype, host=np.ones(n + off, dtype=dtype))
    dr.transform_binary(0, dtype, "plus", buf.at(off), other.at(off), buf.at(off), n)
    assert np.array_equal(buf.numpy()[off:], ((np.arange(n) + 20) * 3 + 1).astype(dtype))
    buf.free()
    other.free()


def test_iota_and_for_each_negate_known_answers(dr):
    """ShpTests.Iota / ForEach (algorithms.cpp:11-37)."""
    g = json.load(open(GOLDEN))
    buf = dr.DeviceArray(0, 10, np.int32)
    dr.iota(0, buf.ptr, 10, g["iota"]["start"], np.int32)
    assert buf.numpy().tolist() == g["iota"]["expected"]
    dr.iota(0, buf.ptr, 10, g["for_each_negate"]["start"], np.int32)
    dr.negate(0, np.int32, buf.ptr, 10)
    assert buf.numpy().tolist() == g["for_each_negate"]["expected"]
    buf.free()


def _halo_exchange(dr, bufs, seg_len, dtype):
    """span_halo exchange (details/halo.hpp:336-387), radius 1, non-periodic:
    first owned cell -> prev rank's next halo, last owned cell -> next rank's
    prev halo; device-to-device copies on the sending segment's stream."""
    it = np.dtype(dtype).itemsize
    P = len(bufs)
    for r in range(P):
        if r > 0:
            dr.d2d(r, bufs[r - 1].at(seg_len + 1), bufs[r].at(1), it)
        if r + 1 < P:
            dr.d2d(r, bufs[r + 1].at(0), bufs[r].at(seg_len), it)
    dr.sync()


@pytest.mark.parametrize("nseg", [1, 2, 3, 4])
def test_stencil1d_known_answer_halo(dr, oracle, nseg):
    """examples/mhp/stencil-1d.cpp: n = 10, 5 steps -> known interior."""
    g = json.load(open(GOLDEN))["stencil_1d"]
    n, steps = g["n"], g["steps"]
    dr.finalize()
    dr.init([0] * nseg)
    try:
        seg = (n + nseg - 1) // nseg
        a = np.arange(g["a_start"], g["a_start"] + n, dtype=np.int32)
        bufs = []
        for which in (a, np.zeros(n, dtype=np.int32)):
            row = []
            for r in range(nseg):
                host = np.zeros(seg + 2, dtype=np.int32)
                part = which[r * seg:(r + 1) * seg]
                host[1:1 + part.size] = part
                row.append(dr.DeviceArray(r, seg + 2, np.int32, host=host))
            bufs.append(row)
        cur = 0
        for _ in range(steps):
            src, dst = bufs[cur], bufs[cur ^ 1]
            _halo_exchange(dr, src, seg, np.int32)
            for r in range(nseg):
                lo = max(0, 1 - r * seg)
                hi = min(seg, n - 1 - r * seg)
                if hi > lo:
                    dr.stencil1d(r, np.int32, src[r].ptr, dst[r].ptr, seg, 1, lo, hi)
            dr.sync()
            cur ^= 1
        res = np.concatenate([bufs[cur][r].numpy()[1:1 + seg] for r in range(nseg)])[:n]
        assert res[1:n - 1].tolist() == g["expected_interior"]
        for row in bufs:
            for b in row:
                b.free()
    finally:
        dr.finalize()
        dr.init([0])


@pytest.mark.parametrize("dtype", [np.float32, np.int32])
@pytest.mark.parametrize("n,r", [(1000, 1), (1001, 1), ((1 << 20) + 3, 1), (5000, 2), (5003, 3), (4099, 4)])
@pytest.mark.parametrize("offset", [0, 1])  # offset 1: unaligned buffers take the scalar kernels
def test_stencil1d_parity(dr, oracle, dtype, n, r, offset):
    rng = np.random.default_rng(n)
    x = (rng.random(n) * 100).astype(dtype) if dtype == np.float32 else rng.integers(-10**6, 10**6, n).astype(dtype)
    src = dr.DeviceArray(0, n + offset, dtype, host=np.concatenate([np.zeros(offset, dtype), x]))
    dst = dr.DeviceArray(0, n + offset, dtype, host=np.zeros(n + offset, dtype))
    isz = np.dtype(dtype).itemsize
    # whole vector = owned region with r halo cells on each side
    dr.stencil1d(0, dtype, src.ptr + offset * isz, dst.ptr + offset * isz, n - 2 * r, r, 0, n - 2 * r)
    ref = oracle.stencil1d(x, r, out=np.zeros(n, dtype))
    got = dst.numpy()[offset:]
    assert np.array_equal(got, ref)  # same left-to-right order from the first term: bit-exact
    src.free()
    dst.free()


@pytest.mark.parametrize("lo,hi", [(0, 0), (5, 6), (3, 700), (123, 997)])
def test_stencil1d_subrange(dr, oracle, lo, hi):
    """Only owned cells [lo, hi) are written (halo.hpp:358-372 owned groups)."""
    n, r = 1000, 1
    x = np.random.default_rng(7).random(n + 2 * r).astype(np.float32)
    src = dr.DeviceArray(0, n + 2 * r, np.float32, host=x)
    dst = dr.DeviceArray(0, n + 2 * r, np.float32, host=np.full(n + 2 * r, -1, np.float32))
    dr.stencil1d(0, np.float32, src.ptr, dst.ptr, n, r, lo, hi)
    ref = oracle.stencil1d(x, r, out=np.zeros(n + 2 * r, np.float32))
    want = np.full(n + 2 * r, -1, np.float32)
    want[r + lo:r + hi] = ref[r + lo:r + hi]
    assert np.array_equal(dst.numpy(), want)
    src.free()
    dst.free()


def test_stencil1d_signed_zero(dr):
    """-0 + -0 + -0 = -0, as the reference's p[-1] + p[0] + p[1] gives."""
    n = 4096
    x = np.full(n, -0.0, np.float32)
    src = dr.DeviceArray(0, n, np.float32, host=x)
    dst = dr.DeviceArray(0, n, np.float32, host=np.ones(n, np.float32))
    dr.stencil1d(0, np.float32, src.ptr, dst.ptr, n - 2, 1, 0, n - 2)
    got = dst.numpy()[1:-1]
    assert np.all(got == 0) and np.all(np.signbit(got))
    src.free()
    dst.free()


@pytest.mark.parametrize("nx,ny", [(513, 300), (512, 300), (1024, 77), (8, 5)])
def test_stencil2d_parity(dr, oracle, nx, ny):
    """5-point row-block stencil (vectorised DPP kernel when nx % 4 == 0)."""
    x = np.random.default_rng(3).random(nx * ny, dtype=np.float32)
    src = dr.DeviceArray(0, nx * ny, np.float32, host=x)
    dst = dr.DeviceArray(0, nx * ny, np.float32, host=x)
    # the whole grid is one row block: halo rows are grid rows 0 and ny-1
    dr.stencil2d(0, np.float32, src.ptr, dst.ptr, nx, ny - 2, 0, ny - 2)
    ref = oracle.stencil2d(x, nx, ny, out=x.copy())
    got = dst.numpy()
    assert np.array_equal(got, ref)  # same summation order as the oracle: bit-exact
    src.free()
    dst.free()


@pytest.mark.parametrize("nx,ny,rlo,rhi", [(2048, 300, 5, 250), (4096, 140, 0, 138), (256, 1000, 63, 64),
                                            (65536, 20, 3, 17)])
def test_stencil2d_row_range(dr, oracle, nx, ny, rlo, rhi):
    """Owned rows [rlo, rhi) of a row block only (the streaming kernel's
    strips of 64 rows, 8-row steps, partial last strip/step); rows outside
    the range keep their old values."""
    x = np.random.default_rng(5).random(nx * ny, dtype=np.float32)
    src = dr.DeviceArray(0, nx * ny, np.float32, host=x)
    dst = dr.DeviceArray(0, nx * ny, np.float32, host=x)
    dr.stencil2d(0, np.float32, src.ptr, dst.ptr, nx, ny - 2, rlo, rhi)
    full = oracle.stencil2d(x, nx, ny, out=x.copy()).reshape(ny, nx)
    want = x.copy().reshape(ny, nx)
    want[1 + rlo:1 + rhi] = full[1 + rlo:1 + rhi]
    assert np.array_equal(dst.numpy().reshape(ny, nx), want)
    src.free()
    dst.free()


@pytest.mark.parametrize("kind", [0, 1])
@pytest.mark.parametrize("m,ncols,row0", [(1000, 1000, 0), (777, 5000, 1234), (1 << 16, 1 << 16, 0)])
def test_csr_generator_matches_oracle(dr, oracle, kind, m, ncols, row0):
    k = 10
    nnz = dr.csr_nnz(kind, row0, m, ncols, k)
    rp = dr.DeviceArray(0, m + 1, np.int32)
    ci = dr.DeviceArray(0, nnz, np.int32)
    va = dr.DeviceArray(0, nnz, np.float32)
    dr.csr_gen(0, kind, row0, m, ncols, k, 42, rp.ptr, ci.ptr, va.ptr)
    orp, oci, ova = oracle.csr_gen("banded" if kind == 0 else "random", row0, m, ncols, 42, k=k)
    assert np.array_equal(rp.numpy(), orp)
    assert np.array_equal(ci.numpy(), oci)
    assert np.array_equal(va.numpy(), ova)
    for b in (rp, ci, va):
        b.free()



@pytest.mark.parametrize("kind", [0, 1])
@pytest.mark.parametrize("m", [1, 1000, 200003])
@pytest.mark.parametrize("vdt,idt", [(np.float32, np.int32), (np.float64, np.int32), (np.float32, np.int64),
                                     (np.float64, np.int64)])
@pytest.mark.parametrize("offset", [0, 1])  # offset 1: colind/vals not vector-aligned -> scalar loads
def test_spmv_parity(dr, oracle, kind, m, vdt, idt, offset):
    """Intended gemv c += A*b (gemv.hpp:13-71), rtol 1e-5 per row vs fp64."""
    ncols = m
    rp, ci, va = oracle.csr_gen("banded" if kind == 0 else "random", 0, m, ncols, 7, k=min(10, ncols))
    x = np.random.default_rng(m).random(ncols).astype(vdt)
    y0 = np.random.default_rng(m + 1).random(m).astype(vdt)
    vav = va.astype(vdt)
    pad = lambda a: np.concatenate([np.zeros(offset, a.dtype), a])
    d = [dr.DeviceArray(0, a.size, a.dtype, host=a) for a in (rp.astype(idt), pad(ci.astype(idt)), pad(vav), x, y0)]
    ci_ptr = d[1].ptr + offset * np.dtype(idt).itemsize
    va_ptr = d[2].ptr + offset * np.dtype(vdt).itemsize
    dr.spmv_csr(0, m, ci.size, d[0].ptr, ci_ptr, va_ptr, d[3].ptr, d[4].ptr,
                vdtype=dr.F32 if vdt == np.float32 else dr.F64, idtype=dr.I32 if idt == np.int32 else dr.I64)
    got = d[4].numpy()
    ref = oracle.csr_spmv(rp, ci, vav, x, y0)
    assert np.max(np.abs(got - ref) / np.maximum(np.abs(ref), 1e-30)) <= (1e-5 if vdt == np.float32 else 1e-12)
    for b in d:
        b.free()


@pytest.mark.parametrize("k", [40, 100, 700])
def test_spmv_long_rows(dr, oracle, k):
    """Rows longer than the CSR-stream limit take the CSR-vector kernel."""
    m = 3001
    rp, ci, va = oracle.csr_gen("random", 0, m, m, 11, k=k)
    x = np.random.default_rng(k).random(m, dtype=np.float32)
    y0 = np.zeros(m, np.float32)
    d = [dr.DeviceArray(0, a.size, a.dtype, host=a) for a in (rp, ci, va, x, y0)]
    dr.spmv_csr(0, m, ci.size, d[0].ptr, d[1].ptr, d[2].ptr, d[3].ptr, d[4].ptr)
    ref = oracle.csr_spmv(rp, ci, va, x, y0)
    assert np.max(np.abs(d[4].numpy() - ref) / np.maximum(np.abs(ref), 1e-30)) <= 1e-5
    for b in d:
        b.free()


@pytest.mark.parametrize("vdt,idt", [(np.float32, np.int32), (np.float64, np.int64), (np.int32, np.int32),
                                     (np.int64, np.int64)])
@pytest.mark.parametrize("m,n,density,row0,rows", [(100, 100, 0.01, 0, 100), (1000, 777, 0.05, 250, 500),
                                                   (64, 5, 0.9, 0, 64), (300, 400, 0.0, 0, 300),
                                                   (5000, 4096, 0.002, 4999, 1)])
def test_csr_gen_density_matches_oracle(dr, oracle, vdt, idt, m, n, density, row0, rows):
    """sparse_matrix(shape, density) generator (sparse_matrix.hpp:157-166) == oracle, bit for bit."""
    nnz = dr.csr_density_nnz(row0, rows, m, n, density)
    orp, oci, ova = oracle.csr_gen_density(row0, rows, m, n, density, 3, int_values=np.dtype(vdt).kind == "i")
    assert nnz == oci.size
    rp = dr.DeviceArray(0, rows + 1, idt)
    ci = dr.DeviceArray(0, max(nnz, 1), idt)
    va = dr.DeviceArray(0, max(nnz, 1), vdt)
    dr.csr_gen_density(0, vdt, idt, row0, rows, m, n, density, 3, rp.ptr, ci.ptr, va.ptr)
    assert np.array_equal(rp.numpy().astype(np.int64), orp)
    assert np.array_equal(ci.numpy()[:nnz].astype(np.int64), oci)
    assert np.array_equal(va.numpy()[:nnz].astype(np.float64), ova)
    for b in (rp, ci, va):
        b.free()


def _irregular_csr(m, seed, long_every=997, long_len=5000):
    """Rows of 0..12 nonzeros, every long_every-th row long_len nonzeros
    (crossing several 2048-slot blocks), sorted unique columns."""
    rng = np.random.default_rng(seed)
    lens = rng.integers(0, 13, m)
    lens[::long_every] = long_len
    lens[1::long_every] = 0
    rp = np.zeros(m + 1, np.int64)
    rp[1:] = np.cumsum(lens)
    ci = np.concatenate([np.sort(rng.choice(m, size=int(k), replace=False)) if k else np.zeros(0, np.int64)
                         for k in lens]).astype(np.int64)
    va = rng.random(ci.size)
    return rp, ci, va


@pytest.mark.parametrize("m", [5000, 100003])
@pytest.mark.parametrize("vdt,idt", [(np.float32, np.int32), (np.float64, np.int64)])
def test_spmv_irregular_rows(dr, oracle, m, vdt, idt):
    """The CSR-stream kernel (average <= 32 nnz/row) on rows of 0..12
    nonzeros with empty rows and long rows spanning several 2048-slot chunks
    (a row block streams its nonzeros chunk by chunk); rtol 1e-5 (f32) /
    1e-12 (f64) per row vs the oracle's sequential CSR (gemv.hpp:13-71,
    intended c += A*b)."""
    rp, ci, va = _irregular_csr(m, m)
    vav = va.astype(vdt)
    x = np.random.default_rng(3).random(m).astype(vdt)
    y0 = np.random.default_rng(4).random(m).astype(vdt)
    d = [dr.DeviceArray(0, a.size, a.dtype, host=a) for a in (rp.astype(idt), ci.astype(idt), vav, x, y0)]
    dr.spmv_csr(0, m, ci.size, d[0].ptr, d[1].ptr, d[2].ptr, d[3].ptr, d[4].ptr,
                vdtype=dr.F32 if vdt == np.float32 else dr.F64, idtype=dr.I32 if idt == np.int32 else dr.I64)
    got = d[4].numpy()
    ref = oracle.csr_spmv(rp.astype(np.int32), ci.astype(np.int32), vav, x, y0)  # the oracle takes int32 indices
    assert np.max(np.abs(got - ref) / np.maximum(np.abs(ref), 1e-30)) <= (1e-5 if vdt == np.float32 else 1e-12)
    for b in d:
        b.free()


@pytest.mark.parametrize("width", [64, 1500, 1840, 2100, 4000])
def test_spmv_band_width_around_x_window(dr, oracle, width):
    """The CSR-stream kernel stages x in an LDS window when a chunk's columns
    span <= 2048 entries and gathers from global memory otherwise (the
    branch is per block): 10 random columns per row inside a band of the
    given width, so blocks fall on both sides of the threshold; f32 / int32
    (the shape that uses the window), rtol 1e-5 per row vs the oracle."""
    m = 300007
    rng = np.random.default_rng(width)
    lo = np.clip(np.arange(m) - width // 2, 0, m - width)
    cols = np.sort(lo[:, None] + np.stack([rng.choice(width, 10, replace=False) for _ in range(64)])[
        np.arange(m) % 64], axis=1)
    rp = (np.arange(m + 1) * 10).astype(np.int32)
    ci = cols.reshape(-1).astype(np.int32)
    va = rng.random(ci.size).astype(np.float32)
    x = rng.random(m).astype(np.float32)
    y0 = rng.random(m).astype(np.float32)
    d = [dr.DeviceArray(0, a.size, a.dtype, host=a) for a in (rp, ci, va, x, y0)]
    dr.spmv_csr(0, m, ci.size, d[0].ptr, d[1].ptr, d[2].ptr, d[3].ptr, d[4].ptr)
    got = d[4].numpy()
    ref = oracle.csr_spmv(rp, ci, va, x, y0)
    assert np.max(np.abs(got - ref) / np.maximum(np.abs(ref), 1e-30)) <= 1e-5
    for b in d:
        b.free()


def _band_csr(m, n, width, shift, seed, anti=False):
    """10 sorted distinct columns per row inside a band of `width` columns
    around the row's scaled diagonal (row i -> i * n / m), moved by `shift`
    (or around the anti-diagonal), clipped to [0, n)."""
    rng = np.random.default_rng(seed)
    d = (np.arange(m, dtype=np.int64) * n) // m
    if anti:
        d = n - 1 - d
    lo = np.clip(d + shift - width // 2, 0, n - width)
    pick = np.stack([np.sort(rng.choice(width, 10, replace=False)) for _ in range(64)])
    ci = (lo[:, None] + pick[np.arange(m) % 64]).reshape(-1)
    rp = np.arange(m + 1, dtype=np.int64) * 10
    return rp, ci, rng.random(ci.size)


@pytest.mark.parametrize("case", ["square_w12", "square_w300", "square_w1500", "shift3000", "anti", "tall", "wide"])
def test_spmv_band_shapes_x_exact_window(dr, oracle, case):
    """The CSR-stream kernel's x windows (speculative from a block's first /
    last column, block min/max) on bands of several widths, a band shifted
    off the diagonal, one on the anti-diagonal (first column > last column
    in every block), tall and wide rectangular matrices; x allocated as
    exactly [min colind, max colind] and passed shifted, as shp::gemv
    passes a tile's window of b (gemv.hpp:34-59 reads b by global column).
    f32 / int32, rtol 1e-5 per row vs the oracle."""
    m = 200003
    if case.startswith("square_w"):
        n, (rp, ci, va) = m, _band_csr(m, m, int(case[8:]), 0, 1)
    elif case == "shift3000":
        n, (rp, ci, va) = m, _band_csr(m, m, 40, 3000, 2)
    elif case == "anti":
        n, (rp, ci, va) = m, _band_csr(m, m, 40, 0, 3, anti=True)
    elif case == "tall":
        n = 50021
        rp, ci, va = _band_csr(m, n, 12, 0, 4)
    else:
        n = 4 * m + 7
        rp, ci, va = _band_csr(m, n, 40, 0, 5)
    rp, ci, va = rp.astype(np.int32), ci.astype(np.int32), va.astype(np.float32)
    x_lo, x_hi = int(ci.min()), int(ci.max()) + 1
    x = np.random.default_rng(11).random(n).astype(np.float32)
    y0 = np.random.default_rng(12).random(m).astype(np.float32)
    d = [dr.DeviceArray(0, a.size, a.dtype, host=a) for a in (rp, ci, va, x[x_lo:x_hi], y0)]
    dr.spmv_csr(0, m, ci.size, d[0].ptr, d[1].ptr, d[2].ptr, d[3].ptr - 4 * x_lo, d[4].ptr)
    got = d[4].numpy()
    for b in d:
        b.free()
    ref = oracle.csr_spmv(rp, ci, va, x, y0)
    assert np.max(np.abs(got - ref) / np.maximum(np.abs(ref), 1e-30)) <= 1e-5


@pytest.mark.parametrize("kind", ["banded", "random"])
@pytest.mark.parametrize("idt", [np.int32, np.int64])
def test_spmv_row_tile_of_larger_matrix(dr, oracle, kind, idt):
    """drhip_spmv_csr on one row tile (global rows [row0, row0 + rows),
    tile-local rowptr) of a 2^22-row matrix with x allocated as exactly the
    tile's column window [lo, hi) and passed shifted -- shp::gemv's call --
    accumulating into a random y; rtol 1e-5 per row vs the oracle's rows."""
    m = 1 << 22
    row0, rows = 1234567, 300001
    orp, oci, ova = oracle.csr_gen(kind, row0, rows, m, 1, k=10)
    lo, hi = int(oci.min()), int(oci.max()) + 1
    x = np.random.default_rng(21).random(m, dtype=np.float32)
    y0 = np.random.default_rng(22).random(rows, dtype=np.float32)
    d = [dr.DeviceArray(0, a.size, a.dtype, host=a) for a in (orp.astype(idt), oci.astype(idt), ova, x[lo:hi], y0)]
    dr.spmv_csr(0, rows, oci.size, d[0].ptr, d[1].ptr, d[2].ptr, d[3].ptr - 4 * lo, d[4].ptr,
                idtype=dr.I32 if idt == np.int32 else dr.I64)
    got = d[4].numpy()
    for b in d:
        b.free()
    ref = oracle.csr_spmv(orp, oci, ova, x, y0)
    assert np.max(np.abs(got - ref) / np.maximum(np.abs(ref), 1e-30)) <= 1e-5
