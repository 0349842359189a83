"""GPU parity: drhip_sort (per-segment LSD radix sort, C-ABI) against the
oracle's sort (oracle.c qsort with std::less comparators).

shp::sort is absent from the reference, so parity is
pinned to std::sort semantics: ascending under std::less.  Keys are
bit-exact (inputs avoid -0.0 and NaN, which std::less leaves unordered)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

DTYPES = [np.uint32, np.int32, np.float32, np.uint64, np.int64, np.float64]


def make_keys(dtype, n, kind, seed):
    rng = np.random.default_rng(seed)
    dt = np.dtype(dtype)
    if kind == "random":
        if dt.kind == "f":
            x = (rng.standard_normal(n) * 1e3).astype(dt)
            x[x == 0] = 1  # no -0.0
            return x
        info = np.iinfo(dt)
        return rng.integers(info.min, info.max, size=n, endpoint=True, dtype=dt)
    if kind == "few":  # low entropy: many equal keys, same digit in most passes
        return rng.integers(0, 5, size=n).astype(dt)
    if kind == "small16":  # small integers: the high digits constant, the low ones uniform
        return rng.integers(0, 1 << 16, size=n).astype(dt)
    if kind == "const":  # every digit constant
        return np.full(n, 12345, dtype=dt)
    if kind == "sorted":
        return np.sort(make_keys(dtype, n, "random", seed))
    if kind == "reversed":
        return np.sort(make_keys(dtype, n, "random", seed))[::-1].copy()
    raise ValueError(kind)


# sort.hip reads DRHIP_SORT_ALGO / DRHIP_SORT_OS_SHAPE at every call: "auto"
# is the shipped policy (onesweep from 256 MiB of keys, classic below); the
# other three force each path so small inputs cover the onesweep kernels too.
# DRHIP_SORT_RANK=ballot forces the ballot ranking that replaces the LDS
# atomic ranking on a device whose ds_add_rtn lane order check fails;
# DRHIP_SORT_STATUS=w64 the 8-byte onesweep status words; DRHIP_SORT_OS_PT=0
# the one-shot onesweep kernel instead of the XCD-grouped persistent one.
ALGOS = {"auto": {}, "classic": {"DRHIP_SORT_ALGO": "classic"},
         "onesweep": {"DRHIP_SORT_ALGO": "onesweep"},
         "onesweep-small": {"DRHIP_SORT_ALGO": "onesweep", "DRHIP_SORT_OS_SHAPE": "small"},
         "classic-ballot": {"DRHIP_SORT_ALGO": "classic", "DRHIP_SORT_RANK": "ballot"},
         "onesweep-ballot": {"DRHIP_SORT_ALGO": "onesweep", "DRHIP_SORT_RANK": "ballot"},
         # 8-byte epoch status words (segments of >= 2^30 keys) at small sizes
         "onesweep-w64": {"DRHIP_SORT_ALGO": "onesweep", "DRHIP_SORT_STATUS": "w64"},
         "onesweep-oneshot": {"DRHIP_SORT_ALGO": "onesweep", "DRHIP_SORT_OS_PT": "0"},
         # a small XCD group: more group boundaries per sort
         "onesweep-group8": {"DRHIP_SORT_ALGO": "onesweep", "DRHIP_SORT_OS_GROUP": "8"},
         # look-back through the agent-scope status copy only
         "onesweep-nolocal": {"DRHIP_SORT_ALGO": "onesweep", "DRHIP_SORT_OS_LOCAL": "0"},
         # fewer per-XCD tile counters than the device's probed XCDs (as on
         # a partitioned part): 3 (not a power of two) and 1 (one sequence)
         "onesweep-nxcd3": {"DRHIP_SORT_ALGO": "onesweep", "DRHIP_SORT_OS_NXCD": "3"},
         "onesweep-nxcd1": {"DRHIP_SORT_ALGO": "onesweep", "DRHIP_SORT_OS_NXCD": "1"}}
ENV_KEYS = sorted({k for v in ALGOS.values() for k in v})


@pytest.fixture(params=list(ALGOS))
def algo(request, monkeypatch):
    for k in ENV_KEYS:
        monkeypatch.delenv(k, raising=False)
    for k, v in ALGOS[request.param].items():
        monkeypatch.setenv(k, v)
    return request.param


def run_sort(dr, x):
    n = x.size
    buf = dr.DeviceArray(0, n, x.dtype, host=x)
    ws = dr.sort_workspace(0, x.dtype, n)
    tmp = dr.DeviceArray(0, max(ws, 16), np.uint8)
    dr.sort_async(0, x.dtype, buf.ptr, n, tmp.ptr, ws)
    got = buf.numpy()
    buf.free()
    tmp.free()
    return got


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("n", [0, 1, 2, 63, 100, 4095, 16384, 65537, (1 << 20) + 13])
def test_sort_random(dr, oracle, algo, dtype, n):
    x = make_keys(dtype, n, "random", seed=n + 1)
    got = run_sort(dr, x)
    assert np.array_equal(got.view(np.uint8), oracle.sort(x).view(np.uint8))


@pytest.mark.parametrize("dtype", [np.uint32, np.int32, np.float32, np.int64])
@pytest.mark.parametrize("kind", ["few", "sorted", "reversed"])
@pytest.mark.parametrize("n", [1000, 300001])
def test_sort_patterns(dr, oracle, algo, dtype, kind, n):
    x = make_keys(dtype, n, kind, seed=7)
    got = run_sort(dr, x)
    assert np.array_equal(got.view(np.uint8), oracle.sort(x).view(np.uint8))


@pytest.mark.parametrize("dtype", [np.uint32, np.float32, np.int64])
@pytest.mark.parametrize("kind", ["small16", "const"])
@pytest.mark.parametrize("n", [(1 << 20) + 13, (1 << 22) + 5])
def test_sort_skewed_digits(dr, oracle, algo, dtype, kind, n):
    """Keys whose high digits are constant (small integers) or all digits
    (one value): whole waves take the one-update fast paths of the ranking
    and of the pre-pass counts (sort.hip kSortUniFast), full and partial
    tiles mixed; bit-exact against the oracle."""
    x = make_keys(dtype, n, kind, 17)
    assert np.array_equal(run_sort(dr, x).view(np.uint8), oracle.sort(x).view(np.uint8))


@pytest.mark.parametrize("dtype", [np.uint32, np.float32, np.int64])
@pytest.mark.parametrize("offset", [1, 2, 3])
@pytest.mark.parametrize("n", [5, 70001])
def test_sort_misaligned_subrange(dr, oracle, algo, dtype, offset, n):
    """A sub-range of a segment (shp::sort over a drop()/subrange): keys
    start off a 16-byte boundary; the elements around it stay untouched."""
    x = make_keys(dtype, n + 2 * offset, "random", seed=n + offset)
    buf = dr.DeviceArray(0, x.size, x.dtype, host=x)
    ws = dr.sort_workspace(0, x.dtype, n)
    tmp = dr.DeviceArray(0, max(ws, 16), np.uint8)
    dr.sort_async(0, x.dtype, buf.at(offset), n, tmp.ptr, ws)
    got = buf.numpy()
    want = x.copy()
    want[offset:offset + n] = oracle.sort(x[offset:offset + n])
    assert np.array_equal(got.view(np.uint8), want.view(np.uint8))
    buf.free()
    tmp.free()


def test_sort_extremes(dr, oracle, algo):
    """Sign bits, extreme values and float specials other than NaN."""
    x = np.array([0, -1, 2**31 - 1, -2**31, 5, -5, 1, -2**31, 0], dtype=np.int32)
    assert np.array_equal(run_sort(dr, x).view(np.uint8), oracle.sort(x).view(np.uint8))
    f = np.array([np.inf, -np.inf, 1e-45, -1e-45, 3.4e38, -3.4e38, 1.0, -1.0, 0.0], np.float32)
    assert np.array_equal(run_sort(dr, f).view(np.uint32), oracle.sort(f).view(np.uint32))


def test_sample_and_bucket_counts(dr, oracle):
    """Distributed-sort helpers: regular samples sorted[j * stride] and
    per-bucket counts of a sorted run against splitters (std::lower_bound
    semantics)."""
    n = 100003
    x = np.sort(make_keys(np.uint32, n, "random", 3))
    buf = dr.DeviceArray(0, n, np.uint32, host=x)
    stride = 6251
    cntn = -(-n // stride)
    smp = dr.DeviceArray(0, cntn, np.uint32)
    dr.sort_sample(0, np.uint32, buf.ptr, n, stride, smp.ptr)
    got = smp.numpy()
    assert cntn == 16 and np.array_equal(got, x[::stride])
    spl = got[[3, 7, 11]].copy()
    sp = dr.DeviceArray(0, 3, np.uint32, host=spl)
    cnt = dr.DeviceArray(0, 4, np.uint64)
    dr.sort_bucket_counts(0, np.uint32, buf.ptr, n, sp.ptr, 3, cnt.ptr)
    lb = np.searchsorted(x, spl, side="left")
    ref = np.diff(np.concatenate([[0], lb, [n]]))
    assert np.array_equal(cnt.numpy(), ref)
    for b in (buf, smp, sp, cnt):
        b.free()


@pytest.mark.parametrize("dtype,n", [(np.uint32, (1 << 26) + 4099), (np.float32, (1 << 26) + 1),
                                     (np.int64, (1 << 25) + 77)])
def test_sort_large_block_shape(dr, algo, dtype, n):
    """Inputs from 256 MiB take the 64 K-key-chunk block shape (sort.hip
    kSortBigBytes); checked against numpy's sort (same std::less order for
    these keys: no NaN, no -0.0), bit for bit."""
    x = make_keys(dtype, n, "random", seed=11)
    got = run_sort(dr, x)
    assert np.array_equal(got.view(np.uint8), np.sort(x).view(np.uint8))


def test_sort_large_few_keys(dr, algo):
    """Low entropy at the large shape: runs of equal digits span sub-tiles and blocks."""
    x = make_keys(np.uint32, (1 << 26) + 5, "few", seed=3)
    got = run_sort(dr, x)
    assert np.array_equal(got, np.sort(x))


def run_merge(dr, x, offs):
    n = x.size
    buf = dr.DeviceArray(0, max(n, 1), x.dtype, host=x if n else np.zeros(1, x.dtype))
    ws = dr.merge_workspace(0, x.dtype, n, len(offs) - 1)
    tmp = dr.DeviceArray(0, max(ws, 16), np.uint8)
    dr.merge_runs(0, x.dtype, buf.ptr, n, offs, tmp.ptr, ws)
    got = buf.numpy()[:n]
    buf.free()
    tmp.free()
    return got


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("sizes", [[1000], [5, 7], [0, 3000, 0], [2048, 2048, 2047, 1], [100000] * 8,
                                   [1, 0, 2, 0, 3, 0, 4, 5000, 9, 77777, 3, 4096, 0, 1, 2, 3, 65536]])
def test_merge_runs(dr, oracle, dtype, sizes):
    """drhip_merge_runs (the distributed sort's destination step): sorted runs -> sorted, bit-exact vs std::sort."""
    runs = [np.sort(make_keys(dtype, s, "random", seed=17 + i)) for i, s in enumerate(sizes)]
    x = np.concatenate(runs) if runs else np.zeros(0, dtype)
    offs = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    got = run_merge(dr, x, offs)
    assert np.array_equal(got.view(np.uint8), oracle.sort(x).view(np.uint8))


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("sizes", [[1000], [5, 7], [0, 3000, 0], [2048, 2048, 2047, 1], [100000] * 8,
                                   [1, 0, 2, 0, 3, 0, 4, 5000, 9, 77777, 3, 4096, 0, 1, 2, 3, 65536]])
@pytest.mark.parametrize("dst_shift", [0, 1])
def test_merge_runs_to(dr, oracle, dtype, sizes, dst_shift):
    """drhip_merge_runs_to: the runs in one buffer (where the distributed
    sort's all_to_all lands) merged straight into another (the segment; a
    sub-range's segment need not be 16-byte aligned): bit-exact vs
    std::sort, src untouched outside its role, nothing written past dst."""
    runs = [np.sort(make_keys(dtype, s, "random", seed=31 + i)) for i, s in enumerate(sizes)]
    x = np.concatenate(runs) if runs else np.zeros(0, dtype)
    n = x.size
    offs = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    sentinel = make_keys(dtype, n + 2, "random", seed=5)
    src = dr.DeviceArray(0, max(n, 1), x.dtype, host=x if n else np.zeros(1, x.dtype))
    dst = dr.DeviceArray(0, n + 2, x.dtype, host=sentinel)
    ws = dr.merge_workspace(0, x.dtype, n, len(offs) - 1)
    tmp = dr.DeviceArray(0, max(ws, 16), np.uint8)
    try:
        dr.merge_runs_to(0, x.dtype, src.ptr, dst.at(dst_shift), n, offs, tmp.ptr, ws)
        got = dst.numpy()
    finally:
        for b in (src, dst, tmp):
            b.free()
    assert np.array_equal(got[dst_shift:dst_shift + n].view(np.uint8), oracle.sort(x).view(np.uint8))
    outside = np.r_[0:dst_shift, dst_shift + n:n + 2]
    assert np.array_equal(got[outside].view(np.uint8), sentinel[outside].view(np.uint8))


@pytest.mark.parametrize("dtype", [np.uint32, np.float32])
def test_merge_runs_ties_and_large(dr, dtype):
    """Many equal keys across runs, 8 runs of 2^22 (the 8-rank shape at 1/64 scale)."""
    runs = [np.sort(make_keys(dtype, 1 << 22, "few", seed=i)) for i in range(8)]
    x = np.concatenate(runs)
    offs = np.arange(9, dtype=np.int64) * (1 << 22)
    got = run_merge(dr, x, offs)
    assert np.array_equal(got, np.sort(x))


def test_sort_concurrent_persistent_on_shared_device(dr, monkeypatch):
    """Three segments on ONE device (duplicated devices, shp-tests.cpp:34-39),
    each >= 256 MiB of keys (the XCD-grouped persistent onesweep), sorted
    without a host sync in between: the per-device ordering lane
    (runtime.hip persistent_lane_*) keeps the resident-grid kernels from
    starving each other; every segment bit-exact vs numpy."""
    for k in ENV_KEYS:
        monkeypatch.delenv(k, raising=False)
    dr.finalize()
    dr.init([0, 0, 0])
    bufs, tmps, xs = [], [], []
    try:
        for seg in range(3):
            n = (1 << 26) + 1000 * seg
            x = make_keys(np.uint32, n, "random", seed=40 + seg)
            ws = dr.sort_workspace(seg, np.uint32, n)
            xs.append(x)
            bufs.append(dr.DeviceArray(seg, n, np.uint32, host=x))
            tmps.append(dr.DeviceArray(seg, ws, np.uint8))
        for seg in range(3):
            dr.sort_async(seg, np.uint32, bufs[seg].ptr, xs[seg].size, tmps[seg].ptr,
                          dr.sort_workspace(seg, np.uint32, xs[seg].size))
        dr.sync()
        for seg in range(3):
            assert np.array_equal(bufs[seg].numpy(), np.sort(xs[seg])), f"segment {seg}"
    finally:
        for b in bufs + tmps:
            b.free()
        dr.finalize()
        dr.init([0])
