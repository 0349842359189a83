"""ctypes binding of libdrhip.so (the C-ABI declared in include/drhip.h).

This is the host-side entry used by the parity tests and by bench.py.  It
calls ONLY the HIP library: there is no CPU fallback, and importing it when
libdrhip.so is missing raises (build it with `make -C distributed-ranges_amd`
or `python -c "import __graft_entry__ as g; g.build()"`).

Device buffers are plain integer addresses (torch tensors' data_ptr(), or
drhip_malloc results); host buffers are numpy arrays.

One HIP runtime per process: the PyTorch-ROCm wheel ships its own
libamdhip64.so / libhsa-runtime64.so (soname without the ".7"), loaded
RTLD_GLOBAL by `import torch`.  When torch is loaded first, libdrhip.so's HIP
symbols bind to that runtime and torch tensors, streams and events mix with
libdrhip calls; when libdrhip.so is loaded first it brings up
/opt/rocm's runtime and a LATER torch import starts a second HIP/HSA runtime
in the process, whose GPU use then fails ("No HIP GPUs are available",
"context is destroyed").  load() therefore imports torch first whenever it
is installed (INTEGRATION.md "one HIP runtime").
"""
import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# DRHIP_LIB selects a variant build (tools/ measurement runs only)
LIB_PATH = os.environ.get("DRHIP_LIB") or os.path.join(HERE, "libdrhip.so")

I32, U32, I64, U64, F32, F64 = 0, 1, 2, 3, 4, 5
PLUS, MUL, MIN, MAX = 0, 1, 2, 3
OPS = {"plus": PLUS, "mul": MUL, "min": MIN, "max": MAX}
DTYPES = {
    np.dtype(np.int32): I32, np.dtype(np.uint32): U32, np.dtype(np.int64): I64,
    np.dtype(np.uint64): U64, np.dtype(np.float32): F32, np.dtype(np.float64): F64,
}
NP_OF = {v: k for k, v in DTYPES.items()}
# accumulation (ACC) numpy type per element dtype code
ACC_OF = {I32: np.int32, U32: np.uint32, I64: np.int64, U64: np.uint64, F32: np.float64,
          F64: np.float64}

# Every exported symbol of include/drhip.h (checked by tests/test_abi.py).
EXPORTS = [
    "drhip_init", "drhip_finalize", "drhip_device_count", "drhip_nprocs", "drhip_device_of",
    "drhip_stream", "drhip_sync", "drhip_sync_all", "drhip_last_error", "drhip_version",
    "drhip_malloc", "drhip_free", "drhip_host_alloc", "drhip_host_free", "drhip_memcpy_h2d",
    "drhip_memcpy_d2h", "drhip_memcpy_d2d", "drhip_fill", "drhip_iota",
    "drhip_transform_scalar", "drhip_transform_binary", "drhip_negate", "drhip_reduce",
    "drhip_dot", "drhip_fold_partials", "drhip_inclusive_scan", "drhip_inclusive_scan_gathered",
    "drhip_reduce_tiles", "drhip_inclusive_scan_tiles", "drhip_spmv_csr", "drhip_csr_nnz", "drhip_csr_gen",
    "drhip_csr_density_nnz", "drhip_csr_gen_density",
    "drhip_sort_workspace", "drhip_sort", "drhip_sort_sample", "drhip_sort_bucket_counts",
    "drhip_split_windows", "drhip_split_exact",
    "drhip_stencil1d", "drhip_stencil2d", "drhip_merge_workspace", "drhip_merge_runs",
    "drhip_merge_runs_to",
    "drhip_comm_unique_id", "drhip_comm_init_rank", "drhip_comm_init_all", "drhip_comm_destroy",
    "drhip_comm_rank", "drhip_comm_group_start", "drhip_comm_group_end", "drhip_allreduce",
    "drhip_allgather", "drhip_gather", "drhip_alltoallv", "drhip_halo_exchange",
    "drhip_graph_begin", "drhip_graph_end", "drhip_graph_launch", "drhip_graph_destroy",
    "drhip_xchg_bytes", "drhip_xchg_alloc", "drhip_xchg_free", "drhip_xchg_allgather", "drhip_ipc_handle",
    "drhip_ipc_open", "drhip_ipc_close",
]

_lib = None


class DrhipError(RuntimeError):
    pass


def load():
    """Load libdrhip.so (raises if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise DrhipError(f"{LIB_PATH} not built: run `make -C {HERE}`")
    try:  # torch's HIP runtime first, so libdrhip binds to it (module docstring)
        import torch  # noqa: F401
    except ImportError:
        pass
    L = C.CDLL(LIB_PATH)
    vp, sz, i, u64 = C.c_void_p, C.c_size_t, C.c_int, C.c_uint64
    sig = {
        "drhip_init": [vp, i], "drhip_finalize": [], "drhip_device_count": [vp],
        "drhip_nprocs": [vp], "drhip_device_of": [i, vp], "drhip_stream": [i, vp],
        "drhip_sync": [i], "drhip_sync_all": [], "drhip_malloc": [i, sz, vp],
        "drhip_free": [i, vp], "drhip_host_alloc": [sz, vp], "drhip_host_free": [vp],
        "drhip_memcpy_h2d": [i, vp, vp, sz], "drhip_memcpy_d2h": [i, vp, vp, sz],
        "drhip_memcpy_d2d": [i, vp, vp, sz], "drhip_fill": [i, vp, sz, vp, sz],
        "drhip_iota": [i, i, vp, sz, vp], "drhip_transform_scalar": [i, i, i, vp, vp, sz, vp],
        "drhip_transform_binary": [i, i, i, vp, vp, vp, sz], "drhip_negate": [i, i, vp, sz],
        "drhip_reduce": [i, i, i, vp, sz, vp], "drhip_dot": [i, i, vp, vp, sz, vp],
        "drhip_fold_partials": [i, i, i, vp, i, i, vp, vp],
        "drhip_inclusive_scan": [i, i, i, vp, vp, sz, vp, vp, vp, vp],
        "drhip_inclusive_scan_gathered": [i, i, i, vp, vp, sz, vp, i, i, vp],
        "drhip_reduce_tiles": [i, i, i, vp, sz, vp],
        "drhip_inclusive_scan_tiles": [i, i, i, vp, vp, sz, vp, vp, i, i, vp],
        "drhip_spmv_csr": [i, i, i, sz, sz, vp, vp, vp, vp, vp],
        "drhip_csr_nnz": [i, sz, sz, sz, i, vp],
        "drhip_csr_gen": [i, i, sz, sz, sz, i, u64, vp, vp, vp],
        "drhip_csr_density_nnz": [sz, sz, sz, sz, C.c_double, vp],
        "drhip_csr_gen_density": [i, i, i, sz, sz, sz, sz, C.c_double, u64, vp, vp, vp],
        "drhip_sort_workspace": [i, i, sz, vp], "drhip_sort": [i, i, vp, sz, vp, sz],
        "drhip_sort_sample": [i, i, vp, sz, sz, vp],
        "drhip_sort_bucket_counts": [i, i, vp, sz, vp, i, vp],
        "drhip_split_windows": [i, vp, vp, vp, vp, i, vp, vp, vp, vp],
        "drhip_split_exact": [i, vp, i, vp, vp, vp, vp, vp, vp],
        "drhip_stencil1d": [i, i, vp, vp, sz, i, sz, sz],
        "drhip_stencil2d": [i, i, vp, vp, sz, sz, sz, sz],
        "drhip_merge_workspace": [i, i, sz, i, vp],
        "drhip_merge_runs": [i, i, vp, sz, vp, i, vp, sz],
        "drhip_merge_runs_to": [i, i, vp, vp, sz, vp, i, vp, sz],
        "drhip_comm_unique_id": [vp], "drhip_comm_init_rank": [i, i, i, vp], "drhip_comm_init_all": [],
        "drhip_comm_destroy": [i], "drhip_comm_rank": [i, vp, vp], "drhip_comm_group_start": [],
        "drhip_comm_group_end": [], "drhip_allreduce": [i, i, i, vp, vp, sz], "drhip_allgather": [i, vp, vp, sz],
        "drhip_gather": [i, vp, vp, sz, i], "drhip_alltoallv": [i, vp, vp, vp, vp, vp, vp],
        "drhip_halo_exchange": [i, vp, sz, sz, sz, sz, i],
        "drhip_graph_begin": [i], "drhip_graph_end": [i, vp], "drhip_graph_launch": [i, vp],
        "drhip_graph_destroy": [vp],
        "drhip_xchg_bytes": [i, vp], "drhip_xchg_alloc": [i, i, vp], "drhip_xchg_free": [i, vp],
        "drhip_xchg_allgather": [i, vp, vp, i, i, vp, i, vp], "drhip_ipc_handle": [vp, vp],
        "drhip_ipc_open": [i, vp, vp], "drhip_ipc_close": [i, vp],
    }
    for name, args in sig.items():
        f = getattr(L, name)
        f.argtypes = args
        f.restype = C.c_int
    L.drhip_last_error.restype = C.c_char_p
    L.drhip_last_error.argtypes = []
    L.drhip_version.restype = C.c_char_p
    L.drhip_version.argtypes = []
    _lib = L
    return L


def check(rc):
    if rc != 0:
        raise DrhipError(f"drhip error {rc}: {load().drhip_last_error().decode()}")


def _hp(a):
    """host pointer of a numpy array (or None)."""
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def _scalar(value, np_type):
    return np.array([value], dtype=np_type)


# ---------------------------------------------------------------- runtime


def device_count():
    n = C.c_int(0)
    rc = load().drhip_device_count(C.byref(n))
    return n.value if rc == 0 else 0


def init(devices):
    devs = (C.c_int * len(devices))(*devices)
    check(load().drhip_init(devs, len(devices)))


def finalize():
    check(load().drhip_finalize())


def nprocs():
    n = C.c_int(0)
    check(load().drhip_nprocs(C.byref(n)))
    return n.value


def stream(seg):
    p = C.c_void_p(0)
    check(load().drhip_stream(seg, C.byref(p)))
    return p.value


def sync(seg=None):
    if seg is None:
        check(load().drhip_sync_all())
    else:
        check(load().drhip_sync(seg))


def graph_begin(seg):
    """Capture the drhip calls that follow on seg's stream (drhip.h)."""
    check(load().drhip_graph_begin(seg))


def graph_end(seg):
    """End the capture; returns the instantiated graph (an opaque handle)."""
    p = C.c_void_p(0)
    check(load().drhip_graph_end(seg, C.byref(p)))
    return p.value


def graph_launch(seg, g):
    check(load().drhip_graph_launch(seg, g))


def graph_destroy(g):
    check(load().drhip_graph_destroy(g))


IPC_HANDLE_BYTES = 64


def xchg_alloc(seg, w):
    """drhip_xchg_alloc: this rank's flag-slot array for w ranks (device
    pointer, fine-grained memory, zeroed)."""
    p = C.c_void_p(0)
    check(load().drhip_xchg_alloc(seg, w, C.byref(p)))
    return p.value


def xchg_free(seg, slots):
    check(load().drhip_xchg_free(seg, slots))


def xchg_allgather(seg, local_slots, peer_slots, rank, value, gathered, value_bytes=8):
    """drhip_xchg_allgather: post the value_bytes (4 / 8) at *value (device)
    to slot `rank` of every array in peer_slots (device pointers valid in
    this process) and gather all w values into gathered[0..w) (device)."""
    arr = (C.c_void_p * len(peer_slots))(*peer_slots)
    check(load().drhip_xchg_allgather(seg, local_slots, arr, len(peer_slots), rank, value, value_bytes, gathered))


def ipc_handle(dev_ptr):
    """drhip_ipc_handle: bytes of the IPC handle of a device allocation."""
    h = (C.c_ubyte * IPC_HANDLE_BYTES)()
    check(load().drhip_ipc_handle(dev_ptr, h))
    return bytes(h)


def ipc_open(seg, handle):
    h = (C.c_ubyte * IPC_HANDLE_BYTES).from_buffer_copy(handle)
    p = C.c_void_p(0)
    check(load().drhip_ipc_open(seg, h, C.byref(p)))
    return p.value


def ipc_close(seg, dev_ptr):
    check(load().drhip_ipc_close(seg, dev_ptr))


def malloc(seg, nbytes):
    p = C.c_void_p(0)
    check(load().drhip_malloc(seg, nbytes, C.byref(p)))
    return p.value


def free(seg, ptr):
    check(load().drhip_free(seg, ptr))


def h2d(seg, dst, arr):
    arr = np.ascontiguousarray(arr)
    check(load().drhip_memcpy_h2d(seg, dst, _hp(arr), arr.nbytes))
    sync(seg)


def d2h(seg, src, count, dtype):
    out = np.empty(count, dtype=dtype)
    if count:
        check(load().drhip_memcpy_d2h(seg, _hp(out), src, out.nbytes))
    sync(seg)
    return out


def d2d(seg, dst, src, nbytes):
    check(load().drhip_memcpy_d2d(seg, dst, src, nbytes))


# ------------------------------------------------------------- algorithms


def fill(seg, dst, n, value, dtype):
    v = _scalar(value, dtype)
    check(load().drhip_fill(seg, dst, n, _hp(v), v.itemsize))


def iota(seg, dst, n, start, dtype):
    v = _scalar(start, dtype)
    check(load().drhip_iota(seg, DTYPES[np.dtype(dtype)], dst, n, _hp(v)))


def transform_scalar(seg, dtype, op, src, dst, n, scalar):
    v = _scalar(scalar, dtype)
    check(load().drhip_transform_scalar(seg, DTYPES[np.dtype(dtype)], OPS[op], src, dst, n, _hp(v)))


def transform_binary(seg, dtype, op, a, b, dst, n):
    check(load().drhip_transform_binary(seg, DTYPES[np.dtype(dtype)], OPS[op], a, b, dst, n))


def negate(seg, dtype, x, n):
    check(load().drhip_negate(seg, DTYPES[np.dtype(dtype)], x, n))


def reduce_async(seg, dtype, op, x, n, out_acc):
    check(load().drhip_reduce(seg, DTYPES[np.dtype(dtype)], OPS[op], x, n, out_acc))


def fold_partials_async(seg, dtype, op, partials, w, rank, result, carry):
    """drhip_fold_partials: left folds of w gathered ACC partials (dtype: a
    numpy dtype or a torch dtype) into *result and, for rank > 0, *carry."""
    try:
        code = DTYPES[np.dtype(dtype)]
    except TypeError:
        code = DTYPES[np.dtype(str(dtype).replace("torch.", ""))]
    check(load().drhip_fold_partials(seg, code, OPS[op], partials, w, rank, result or None, carry or None))


def dot_async(seg, dtype, x, y, n, out_acc):
    check(load().drhip_dot(seg, DTYPES[np.dtype(dtype)], x, y, n, out_acc))


def scan_async(seg, dtype, op, src, dst, n, init=None, carry=None, carry_dev=None, total_dev=None):
    code = DTYPES[np.dtype(dtype)]
    iv = None if init is None else _scalar(init, dtype)
    cv = None if carry is None else _scalar(carry, ACC_OF[code])
    check(load().drhip_inclusive_scan(seg, code, OPS[op], src, dst, n, _hp(iv), _hp(cv),
                                      carry_dev, total_dev))


def scan_gathered_async(seg, dtype, op, src, dst, n, partials, w, rank, result=None):
    """drhip_inclusive_scan_gathered: scan with the carry folded from the w
    gathered partials (ranks < rank) and *result = the fold of all w."""
    check(load().drhip_inclusive_scan_gathered(seg, DTYPES[np.dtype(dtype)], OPS[op], src, dst, n, partials, w, rank,
                                               result or None))


def reduce_tiles_async(seg, dtype, op, x, n, out_acc):
    """drhip_reduce_tiles: drhip_reduce that also leaves the scan tiles'
    prefixes for a following scan_tiles_async over the same range."""
    check(load().drhip_reduce_tiles(seg, DTYPES[np.dtype(dtype)], OPS[op], x, n, out_acc))


def scan_tiles_async(seg, dtype, op, src, dst, n, carry_dev=None, partials=None, w=0, rank=0, result=None):
    """drhip_inclusive_scan_tiles: the scan of the range the segment's last
    reduce_tiles_async reduced, from its tile prefixes (no look-back)."""
    check(load().drhip_inclusive_scan_tiles(seg, DTYPES[np.dtype(dtype)], OPS[op], src, dst, n, carry_dev or None,
                                            partials or None, w, rank, result or None))


def spmv_csr(seg, m, nnz, rowptr, colind, vals, x, y, vdtype=F32, idtype=I32):
    check(load().drhip_spmv_csr(seg, vdtype, idtype, m, nnz, rowptr, colind, vals, x, y))


def csr_nnz(kind, row0, nrows, ncols, k=10):
    out = C.c_size_t(0)
    check(load().drhip_csr_nnz(kind, row0, nrows, ncols, k, C.byref(out)))
    return out.value


def csr_gen(seg, kind, row0, nrows, ncols, k, seed, rowptr, colind, vals):
    check(load().drhip_csr_gen(seg, kind, row0, nrows, ncols, k, seed, rowptr, colind, vals))


def csr_density_nnz(row0, nrows, m, ncols, density):
    out = C.c_size_t(0)
    check(load().drhip_csr_density_nnz(row0, nrows, m, ncols, density, C.byref(out)))
    return out.value


def csr_gen_density(seg, vdtype, idtype, row0, nrows, m, ncols, density, seed, rowptr, colind, vals):
    check(load().drhip_csr_gen_density(seg, DTYPES[np.dtype(vdtype)], DTYPES[np.dtype(idtype)], row0, nrows, m,
                                       ncols, density, seed, rowptr, colind, vals))


def merge_workspace(seg, dtype, n, nruns):
    out = C.c_size_t(0)
    check(load().drhip_merge_workspace(seg, DTYPES[np.dtype(dtype)], n, nruns, C.byref(out)))
    return out.value


def merge_runs(seg, dtype, keys, n, run_offsets, tmp, tmp_bytes):
    """Sort keys[0, n) made of sorted runs [run_offsets[r], run_offsets[r+1])."""
    offs = (C.c_size_t * len(run_offsets))(*[int(o) for o in run_offsets])
    check(load().drhip_merge_runs(seg, DTYPES[np.dtype(dtype)], keys, n, offs, len(run_offsets) - 1, tmp, tmp_bytes))


def merge_runs_to(seg, dtype, src, dst, n, run_offsets, tmp, tmp_bytes):
    """dst[0, n) = the merge of src's sorted runs [run_offsets[r], run_offsets[r+1])."""
    offs = (C.c_size_t * len(run_offsets))(*[int(o) for o in run_offsets])
    check(load().drhip_merge_runs_to(seg, DTYPES[np.dtype(dtype)], src, dst, n, offs, len(run_offsets) - 1, tmp,
                                     tmp_bytes))


def sort_workspace(seg, dtype, n):
    out = C.c_size_t(0)
    check(load().drhip_sort_workspace(seg, DTYPES[np.dtype(dtype)], n, C.byref(out)))
    return out.value


def sort_async(seg, dtype, keys, n, tmp, tmp_bytes):
    check(load().drhip_sort(seg, DTYPES[np.dtype(dtype)], keys, n, tmp, tmp_bytes))


def sort_sample(seg, dtype, sorted_ptr, n, stride, samples):
    """samples[j] = sorted[j * stride], j < ceil(n / stride)."""
    check(load().drhip_sort_sample(seg, DTYPES[np.dtype(dtype)], sorted_ptr, n, stride, samples))


def _u64(a):
    return np.ascontiguousarray(a, dtype=np.uint64)


def split_windows(n, stride, nsamples, samples, g):
    """Host step of the distributed sort's exact splitting (csrc/split.hip,
    no GPU needed): per boundary g[k] the bracket (lo, hi) and win[p, nb, 2]
    = each rank's slice [a, b) of its sorted keys holding the bracket."""
    n, stride, nsamples, samples, g = map(_u64, (n, stride, nsamples, samples, g))
    p, nb = n.size, g.size
    lo, hi = np.zeros(max(nb, 1), np.uint64), np.zeros(max(nb, 1), np.uint64)
    win = np.zeros((p, max(nb, 1), 2), np.uint64)
    check(load().drhip_split_windows(p, _hp(n), _hp(stride), _hp(nsamples), _hp(samples) if samples.size else None,
                                     nb, _hp(g), _hp(lo), _hp(hi), _hp(win)))
    return lo[:nb], hi[:nb], win[:, :nb]


def split_exact(n, g, lo, hi, win, wkeys):
    """split[p, nb + 1]: rank i's keys going to destinations <= k (exact)."""
    n, g, lo, hi, wkeys = map(_u64, (n, g, lo, hi, wkeys))
    win = _u64(win)
    p, nb = n.size, g.size
    split = np.zeros((p, nb + 1), np.uint64)
    check(load().drhip_split_exact(p, _hp(n), nb, _hp(g), _hp(lo), _hp(hi), _hp(win),
                                   _hp(wkeys) if wkeys.size else None, _hp(split)))
    return split


def sort_bucket_counts(seg, dtype, sorted_ptr, n, splitters, nsplit, counts):
    check(load().drhip_sort_bucket_counts(seg, DTYPES[np.dtype(dtype)], sorted_ptr, n, splitters,
                                          nsplit, counts))


def stencil1d(seg, dtype, in_buf, out_buf, n_owned, radius, lo, hi):
    check(load().drhip_stencil1d(seg, DTYPES[np.dtype(dtype)], in_buf, out_buf, n_owned, radius,
                                 lo, hi))


def stencil2d(seg, dtype, in_buf, out_buf, nx, rows, rlo, rhi):
    check(load().drhip_stencil2d(seg, DTYPES[np.dtype(dtype)], in_buf, out_buf, nx, rows, rlo, rhi))


# ------------------------------------------------ RCCL over xGMI (comm.hip)
COMM_ID_BYTES = 128


def comm_unique_id():
    """128-byte RCCL unique id (rank 0 makes it, every rank receives it)."""
    buf = C.create_string_buffer(COMM_ID_BYTES)
    check(load().drhip_comm_unique_id(buf))
    return buf.raw


def comm_init_rank(seg, nranks, rank, uid):
    check(load().drhip_comm_init_rank(seg, nranks, rank, C.create_string_buffer(bytes(uid), COMM_ID_BYTES)))


def comm_init_all():
    check(load().drhip_comm_init_all())


def comm_destroy(seg):
    check(load().drhip_comm_destroy(seg))


def comm_rank(seg):
    r, n = C.c_int(), C.c_int()
    check(load().drhip_comm_rank(seg, C.byref(r), C.byref(n)))
    return r.value, n.value


def allreduce(seg, dtype, op, send, recv, n):
    check(load().drhip_allreduce(seg, DTYPES[np.dtype(dtype)], OPS[op], send, recv, n))


def allgather(seg, send, recv, nbytes):
    check(load().drhip_allgather(seg, send, recv, nbytes))


def gather(seg, send, recv, nbytes, root):
    check(load().drhip_gather(seg, send, recv, nbytes, root))


def alltoallv(seg, send, send_bytes, send_off, recv, recv_bytes, recv_off):
    a = [np.ascontiguousarray(v, dtype=np.uint64) for v in (send_bytes, send_off, recv_bytes, recv_off)]
    check(load().drhip_alltoallv(seg, send, _hp(a[0]), _hp(a[1]), recv, _hp(a[2]), _hp(a[3])))


def halo_exchange(seg, buf, n_owned, cell_bytes, prev, nxt, periodic=False):
    check(load().drhip_halo_exchange(seg, buf, n_owned, cell_bytes, prev, nxt, int(periodic)))


# ------------------------------------------------ convenience (host arrays)


class DeviceArray:
    """A device buffer on one segment, filled from / read back to numpy."""

    def __init__(self, seg, count, dtype, host=None):
        self.seg, self.count, self.dtype = seg, int(count), np.dtype(dtype)
        self.nbytes = self.count * self.dtype.itemsize
        self.ptr = malloc(seg, max(self.nbytes, 16))
        sync(seg)
        if host is not None:
            h2d(seg, self.ptr, np.ascontiguousarray(host, dtype=self.dtype))

    def at(self, offset):
        return self.ptr + offset * self.dtype.itemsize

    def numpy(self):
        return d2h(self.seg, self.ptr, self.count, self.dtype)

    def free(self):
        if self.ptr:
            free(self.seg, self.ptr)
            sync(self.seg)
            self.ptr = 0


def reduce(seg, x_ptr, n, dtype, op="plus"):
    """Reduce n elements at device address x_ptr; returns the ACC value."""
    code = DTYPES[np.dtype(dtype)]
    out = DeviceArray(seg, 1, ACC_OF[code])
    reduce_async(seg, dtype, op, x_ptr, n, out.ptr)
    r = out.numpy()[0]
    out.free()
    return r
