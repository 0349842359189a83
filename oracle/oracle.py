"""ctypes binding of the CPU oracle (oracle/liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, never by the product path.  See oracle.h for
the reference file:line each function restates.
"""
import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

PLUS, MUL, MIN, MAX = 0, 1, 2, 3
OPS = {"plus": PLUS, "mul": MUL, "min": MIN, "max": MAX}

_CT = {
    "i32": (np.int32, C.c_int32),
    "u32": (np.uint32, C.c_uint32),
    "i64": (np.int64, C.c_int64),
    "u64": (np.uint64, C.c_uint64),
    "f32": (np.float32, C.c_float),
    "f64": (np.float64, C.c_double),
}


def build():
    import subprocess
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _LIB
    if _LIB is None:
        # ORACLE_LIB: the sanitizer build (oracle/Makefile `asan`, driven by
        # tests/test_sanitize.py); the default is the optimised library
        path = os.environ.get("ORACLE_LIB") or os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            build()
        _LIB = C.CDLL(path)
        _setup(_LIB)
    return _LIB


def _p(a):
    return a.ctypes.data_as(C.c_void_p) if a is not None else None


def _setup(L):
    vp, sz, i = C.c_void_p, C.c_size_t, C.c_int
    L.orc_dv_segments.argtypes = [sz, i, vp]
    L.orc_dv_segments.restype = i
    L.orc_subrange_segments.argtypes = [vp, i, sz, sz, vp, vp]
    L.orc_subrange_segments.restype = i
    L.orc_zip_pieces.argtypes = [vp, i, vp, i, vp, vp, vp, i]
    L.orc_zip_pieces.restype = i
    for suf, (_, ct) in _CT.items():
        f = getattr(L, "orc_shp_reduce_" + suf)
        f.argtypes = [vp, vp, i, ct, i]
        f.restype = ct
        g = getattr(L, "orc_shp_scan_" + suf)
        g.argtypes = [vp, vp, vp, i, i, i, ct]
        g.restype = None
    L.orc_reduce_exact_f32.argtypes = [vp, sz, C.c_double, i]
    L.orc_reduce_exact_f32.restype = C.c_double
    L.orc_reduce_exact_f64.argtypes = [vp, sz, C.c_double, i]
    L.orc_reduce_exact_f64.restype = C.c_double
    L.orc_dot_f32.argtypes = [vp, vp, sz, C.c_double]
    L.orc_dot_f32.restype = C.c_double
    L.orc_dot_f64.argtypes = [vp, vp, sz, C.c_double]
    L.orc_dot_f64.restype = C.c_double
    L.orc_dot_i32.argtypes = [vp, vp, sz, C.c_int32]
    L.orc_dot_i32.restype = C.c_int32
    L.orc_scan_exact_f32.argtypes = [vp, vp, sz, i, i, C.c_double]
    L.orc_mhp_reduce_f32.argtypes = [vp, sz, i, C.c_double, i]
    L.orc_mhp_reduce_f32.restype = C.c_double
    L.orc_mhp_reduce_i32.argtypes = [vp, sz, i, C.c_int32, i]
    L.orc_mhp_reduce_i32.restype = C.c_int32
    L.orc_mhp_scan_f32.argtypes = [vp, vp, sz, i, i]
    L.orc_mhp_scan_i32.argtypes = [vp, vp, sz, i, i]
    L.orc_csr_spmv_f32_i32.argtypes = [sz, vp, vp, vp, vp, vp, vp]
    L.orc_csr_spmv_f64_i32.argtypes = [sz, vp, vp, vp, vp, vp, vp]
    L.orc_csr_banded_nnz.argtypes = [sz, sz]
    L.orc_csr_banded_nnz.restype = sz
    L.orc_csr_gen_banded_f32.argtypes = [sz, sz, sz, C.c_uint64, vp, vp, vp]
    L.orc_csr_gen_random_f32.argtypes = [sz, sz, sz, i, C.c_uint64, vp, vp, vp]
    L.orc_u01.argtypes = [C.c_uint64, C.c_uint64, C.c_uint64]
    L.orc_u01.restype = C.c_float
    L.orc_hash3.argtypes = [C.c_uint64, C.c_uint64, C.c_uint64]
    L.orc_hash3.restype = C.c_uint64
    L.orc_sort_u32.argtypes = [vp, sz]
    L.orc_radix_sort_u32.argtypes = [vp, sz]
    L.orc_radix_sort_u32.restype = i
    L.orc_radix_sort_u32_par.argtypes = [vp, sz, i]
    L.orc_radix_sort_u32_par.restype = i
    L.orc_fill_hash_u32.argtypes = [vp, sz, C.c_uint64, C.c_uint64, i]
    L.orc_sort_i32.argtypes = [vp, sz]
    L.orc_sort_f32.argtypes = [vp, sz]
    L.orc_sort_u64.argtypes = [vp, sz]
    L.orc_sort_i64.argtypes = [vp, sz]
    L.orc_sort_f64.argtypes = [vp, sz]
    L.orc_stencil1d_i32.argtypes = [vp, vp, sz, i]
    L.orc_stencil1d_f32.argtypes = [vp, vp, sz, i]
    L.orc_stencil1d_mhp_steps_i32.argtypes = [vp, vp, sz, i, i]
    L.orc_stencil1d_mhp_steps_i32.restype = i
    L.orc_stencil_mhp_test_op_i32.argtypes = [vp, vp, sz, i]
    L.orc_stencil2d_f32.argtypes = [vp, vp, sz, sz]
    L.orc_csr_density_nnz.argtypes = [sz, sz, sz, sz, C.c_double]
    L.orc_csr_density_nnz.restype = sz
    L.orc_csr_gen_density.argtypes = [sz, sz, sz, sz, C.c_double, C.c_uint64, i, vp, vp, vp]
    L.orc_lrand48_mod.argtypes = [vp, sz, C.c_int32, i]


# ---------------------------------------------------------------- helpers


def dv_segments(n, nprocs):
    out = np.zeros(max(nprocs, 1), dtype=np.uintp)
    k = lib().orc_dv_segments(n, nprocs, _p(out))
    return [int(v) for v in out[:k]]


def subrange_segments(lens, b, e):
    ln = np.asarray(lens, dtype=np.uintp)
    out = np.zeros(len(lens), dtype=np.uintp)
    rk = np.zeros(len(lens), dtype=np.int32)
    k = lib().orc_subrange_segments(_p(ln), len(lens), b, e, _p(out), _p(rk))
    return [int(v) for v in out[:k]], [int(v) for v in rk[:k]]


def zip_pieces(lens_r, lens_o):
    a = np.asarray(lens_r, dtype=np.uintp)
    b = np.asarray(lens_o, dtype=np.uintp)
    cap = len(lens_r) + len(lens_o) + 1
    out = np.zeros(cap, dtype=np.uintp)
    rr = np.zeros(cap, dtype=np.int32)
    ro = np.zeros(cap, dtype=np.int32)
    k = lib().orc_zip_pieces(_p(a), len(a), _p(b), len(b), _p(out), _p(rr), _p(ro), cap)
    return [int(v) for v in out[:k]], [int(v) for v in rr[:k]], [int(v) for v in ro[:k]]


def _suffix(arr):
    for suf, (npt, _) in _CT.items():
        if arr.dtype == npt:
            return suf
    raise TypeError(arr.dtype)


def shp_reduce(x, seg_lens, init, op="plus"):
    x = np.ascontiguousarray(x)
    suf = _suffix(x)
    ln = np.asarray(seg_lens, dtype=np.uintp)
    f = getattr(lib(), "orc_shp_reduce_" + suf)
    return f(_p(x), _p(ln), len(ln), _CT[suf][0](init).item(), OPS[op])


def shp_scan(x, pieces, op="plus", init=None):
    x = np.ascontiguousarray(x)
    suf = _suffix(x)
    out = np.empty_like(x)
    pc = np.asarray(pieces, dtype=np.uintp)
    f = getattr(lib(), "orc_shp_scan_" + suf)
    f(_p(x), _p(out), _p(pc), len(pc), OPS[op], int(init is not None),
      _CT[suf][0](0 if init is None else init).item())
    return out


def reduce_exact(x, init=0.0, op="plus"):
    x = np.ascontiguousarray(x)
    if x.dtype == np.float32:
        return lib().orc_reduce_exact_f32(_p(x), x.size, float(init), OPS[op])
    return lib().orc_reduce_exact_f64(_p(np.ascontiguousarray(x, dtype=np.float64)),
                                      x.size, float(init), OPS[op])


def scan_exact_f32(x, op="plus", init=None):
    x = np.ascontiguousarray(x, dtype=np.float32)
    out = np.empty(x.size, dtype=np.float64)
    lib().orc_scan_exact_f32(_p(x), _p(out), x.size, OPS[op], int(init is not None),
                             float(0.0 if init is None else init))
    return out


def dot(x, y, init=0):
    x = np.ascontiguousarray(x)
    y = np.ascontiguousarray(y)
    if x.dtype == np.float32:
        return lib().orc_dot_f32(_p(x), _p(y), x.size, float(init))
    if x.dtype == np.float64:
        return lib().orc_dot_f64(_p(x), _p(y), x.size, float(init))
    return lib().orc_dot_i32(_p(x), _p(y), x.size, int(init))


def mhp_reduce_f32(x, nranks, init=0.0, nthreads=1):
    x = np.ascontiguousarray(x, dtype=np.float32)
    return lib().orc_mhp_reduce_f32(_p(x), x.size, nranks, float(init), nthreads)


def mhp_reduce_i32(x, nranks, init=0, nthreads=1):
    x = np.ascontiguousarray(x, dtype=np.int32)
    return lib().orc_mhp_reduce_i32(_p(x), x.size, nranks, int(init), nthreads)


def mhp_scan(x, nranks, nthreads=1, out=None):
    x = np.ascontiguousarray(x)
    if out is None:
        out = np.empty_like(x)
    if x.dtype == np.float32:
        lib().orc_mhp_scan_f32(_p(x), _p(out), x.size, nranks, nthreads)
    else:
        lib().orc_mhp_scan_i32(_p(x), _p(out), x.size, nranks, nthreads)
    return out


def csr_spmv(rowptr, colind, vals, x, y_in=None):
    m = rowptr.size - 1
    out = np.empty(m, dtype=np.float64)
    f = lib().orc_csr_spmv_f32_i32 if vals.dtype == np.float32 else lib().orc_csr_spmv_f64_i32
    f(m, _p(rowptr), _p(colind), _p(vals), _p(x), _p(y_in), _p(out))
    return out


def csr_gen_density(row0, nrows, m, ncols, density, seed, int_values=False):
    """Rows [row0, row0+nrows) of the density generator (int64 rowptr/colind, float64 values)."""
    L = lib()
    nnz = L.orc_csr_density_nnz(row0, nrows, m, ncols, density)
    rowptr = np.empty(nrows + 1, dtype=np.int64)
    colind = np.empty(max(nnz, 1), dtype=np.int64)
    vals = np.empty(max(nnz, 1), dtype=np.float64)
    L.orc_csr_gen_density(row0, nrows, m, ncols, density, seed, int(int_values), _p(rowptr), _p(colind), _p(vals))
    return rowptr, colind[:nnz], vals[:nnz]


def csr_gen(kind, row0, nrows, ncols, seed, k=10):
    L = lib()
    if kind == "banded":
        nnz = L.orc_csr_banded_nnz(row0 + nrows, ncols) - L.orc_csr_banded_nnz(row0, ncols)
    else:
        nnz = nrows * min(k, ncols)
    rowptr = np.empty(nrows + 1, dtype=np.int32)
    colind = np.empty(max(nnz, 1), dtype=np.int32)
    vals = np.empty(max(nnz, 1), dtype=np.float32)
    if kind == "banded":
        L.orc_csr_gen_banded_f32(row0, nrows, ncols, seed, _p(rowptr), _p(colind), _p(vals))
    else:
        L.orc_csr_gen_random_f32(row0, nrows, ncols, k, seed, _p(rowptr), _p(colind), _p(vals))
    return rowptr, colind[:nnz], vals[:nnz]


def sort(x):
    x = np.array(x, copy=True)
    f = {np.dtype(np.uint32): lib().orc_sort_u32, np.dtype(np.int32): lib().orc_sort_i32,
         np.dtype(np.float32): lib().orc_sort_f32, np.dtype(np.uint64): lib().orc_sort_u64,
         np.dtype(np.int64): lib().orc_sort_i64, np.dtype(np.float64): lib().orc_sort_f64}[x.dtype]
    f(_p(x), x.size)
    return x


def sort_u32_large(x):
    """std::sort order of uint32 keys in O(n) (orc_radix_sort_u32), for the
    full-size C3 checks; pinned to the qsort form in tests/test_oracle.py."""
    x = np.array(x, dtype=np.uint32, copy=True)
    if lib().orc_radix_sort_u32(_p(x), x.size) != 0:
        raise MemoryError("orc_radix_sort_u32")
    return x


def sort_u32_large_par(x, threads=8):
    """orc_radix_sort_u32's output from OpenMP passes (orc_radix_sort_u32_par)."""
    x = np.array(x, dtype=np.uint32, copy=True)
    if lib().orc_radix_sort_u32_par(_p(x), x.size, threads) != 0:
        raise MemoryError("orc_radix_sort_u32_par")
    return x


def hash_u32(n, seed, start=0, threads=8):
    """The synthetic C3 keys: high 32 bits of splitmix64(seed + start + i)."""
    x = np.empty(n, np.uint32)
    lib().orc_fill_hash_u32(_p(x), n, seed, start, threads)
    return x


def stencil1d(x, radius=1, out=None):
    x = np.ascontiguousarray(x)
    if out is None:
        out = np.array(x, copy=True)
    f = lib().orc_stencil1d_i32 if x.dtype == np.int32 else lib().orc_stencil1d_f32
    f(_p(x), _p(out), x.size, radius)
    return out


def stencil1d_mhp_steps(a, b, nranks, steps):
    a = np.array(a, dtype=np.int32, copy=True)
    b = np.array(b, dtype=np.int32, copy=True)
    cur = lib().orc_stencil1d_mhp_steps_i32(_p(a), _p(b), a.size, nranks, steps)
    return a, b, cur


def stencil_mhp_test_op(x, radius, out):
    x = np.ascontiguousarray(x, dtype=np.int32)
    lib().orc_stencil_mhp_test_op_i32(_p(x), _p(out), x.size, radius)
    return out


def stencil2d(x, nx, ny, out=None):
    x = np.ascontiguousarray(x, dtype=np.float32)
    if out is None:
        out = np.array(x, copy=True)
    lib().orc_stencil2d_f32(_p(x), _p(out), nx, ny)
    return out


def lrand48_mod(n, mod=100, reseed=False):
    out = np.empty(n, dtype=np.int32)
    lib().orc_lrand48_mod(_p(out), n, mod, int(reseed))
    return out
