"""GPU parity at the BASELINE.json configs' REAL sizes, each
through the C-ABI and checked against the oracle (oracle/liboracle.so):

  C2  reduce + inclusive_scan, 2^30 fp32 U[0,1): rel <= 1e-5 (reduce) and per
      element rel <= 1e-5 vs the fp64 prefix (scan); 2^30 int32 U[0,2^16):
      bit-exact vs oracle.shp_reduce / shp_scan (wrapping), on 1 segment and
      on the 8-segment distributed form (carries between segments).
  C3  sort of 2^28 uint32 keys (one GPU's share of 2^31 over 8): the same
      bytes as the oracle's std::sort-order sort, i.e. sorted AND a
      permutation of the input.
  C4  CSR gemv, 2^26 x 2^26, ~10 nnz/row, banded and random (the device
      generator): rows rel <= 1e-5 vs fp64 rows rebuilt by the oracle's
      row-addressable generator, on windows covering both ends, the 8-way
      row-tile edges and random interior rows; plus one 1/8 row tile.
  C5  1-D 3-point stencil on 2^29 cells and 2-D 5-point on 8192 x 65536
      cells (one GPU's share of 2^32 over 8): every cell bit-exact vs the
      oracle (same left-to-right summation order); 1-D with 8 segments and
      halo exchanges for 3 steps, every cell bit-exact.

The reference's own tests are far smaller (n <= 200, test/gtest/shp/
algorithms.cpp:39-149); these pin the same algorithms at the sizes the bench
reports."""
import numpy as np
import pytest

from test_gpu_scan import shp_scan_via_abi

pytestmark = pytest.mark.gpu

FP_RTOL = 1e-5
N30 = 1 << 30


def max_rel_err(got, ref, chunk=1 << 26):
    """max |got - ref| / |ref| over all elements, chunked (8 GiB fp64 refs)."""
    err = 0.0
    for i in range(0, ref.size, chunk):
        r = ref[i:i + chunk]
        g = got[i:i + chunk].astype(np.float64)
        err = max(err, float(np.max(np.abs(g - r) / np.maximum(np.abs(r), 1e-30))))
    return err


# ------------------------------------------------------------------ C2

def test_c2_reduce_scan_f32_2pow30(dr, oracle):
    x = np.random.default_rng(1).random(N30, dtype=np.float32)
    src = dr.DeviceArray(0, N30, np.float32, host=x)
    dst = dr.DeviceArray(0, N30, np.float32)
    try:
        got_r = float(dr.reduce(0, src.ptr, N30, np.float32))
        ref_r = oracle.reduce_exact(x)
        assert abs(got_r - ref_r) / ref_r <= FP_RTOL
        dr.scan_async(0, np.float32, "plus", src.ptr, dst.ptr, N30)
        got = dst.numpy()
        ref = oracle.scan_exact_f32(x)
        assert max_rel_err(got, ref) <= FP_RTOL
        # the scan's last element and the reduce agree (the bench's cheap check)
        assert abs(float(got[-1]) - got_r) / got_r <= FP_RTOL
    finally:
        src.free()
        dst.free()


@pytest.mark.parametrize("dtype", [np.float32, np.int32])
def test_c2_reduce_tiles_scan_tiles_2pow30(dr, oracle, dtype):
    """C2 at 2^30 through the step the bench runs: drhip_reduce_tiles (the
    reduce, leaving the scan tiles' prefixes) then drhip_inclusive_scan_tiles
    (the scan without look-back).  fp32: reduce rel <= 1e-5 vs fp64, every
    element rel <= 1e-5 vs the fp64 prefix; int32: bit-exact vs the oracle."""
    if dtype == np.float32:
        x = np.random.default_rng(11).random(N30, dtype=np.float32)
    else:
        x = np.random.default_rng(11).integers(0, 1 << 16, N30, dtype=np.int32)
    acc = np.float64 if dtype == np.float32 else np.int32
    src = dr.DeviceArray(0, N30, dtype, host=x)
    dst = dr.DeviceArray(0, N30, dtype)
    red = dr.DeviceArray(0, 1, acc)
    try:
        dr.reduce_tiles_async(0, dtype, "plus", src.ptr, N30, red.ptr)
        dr.scan_tiles_async(0, dtype, "plus", src.ptr, dst.ptr, N30)
        got_r = red.numpy()[0]
        got = dst.numpy()
    finally:
        src.free()
        dst.free()
        red.free()
    if dtype == np.float32:
        ref_r = oracle.reduce_exact(x)
        assert abs(float(got_r) - ref_r) / ref_r <= FP_RTOL
        assert max_rel_err(got, oracle.scan_exact_f32(x)) <= FP_RTOL
    else:
        assert int(got_r) == int(oracle.shp_reduce(x, [N30], 0))
        assert np.array_equal(got, oracle.shp_scan(x, [N30], "plus"))


def test_c2_reduce_scan_i32_2pow30_bit_exact(dr, oracle):
    x = np.random.default_rng(1).integers(0, 1 << 16, N30, dtype=np.int32)
    src = dr.DeviceArray(0, N30, np.int32, host=x)
    dst = dr.DeviceArray(0, N30, np.int32)
    try:
        assert int(dr.reduce(0, src.ptr, N30, np.int32)) == int(oracle.shp_reduce(x, [N30], 0))
        dr.scan_async(0, np.int32, "plus", src.ptr, dst.ptr, N30)
        assert np.array_equal(dst.numpy(), oracle.shp_scan(x, [N30], "plus"))
    finally:
        src.free()
        dst.free()


def test_c2_scan_i32_2pow30_eight_segments(dr, oracle):
    """The 8-GPU form of C2 (2^27 per segment), run as 8 segments of one GPU:
    per-segment totals, carries, carry-in scans -- bit-exact with the
    reference's 3-phase algorithm (oracle.shp_scan over the same pieces)."""
    x = np.random.default_rng(2).integers(0, 1 << 16, N30, dtype=np.int32)
    dr.finalize()
    dr.init([0] * 8)
    try:
        got = shp_scan_via_abi(dr, oracle, x, N30, 8, "plus", None)
    finally:
        dr.finalize()
        dr.init([0])
    assert np.array_equal(got, oracle.shp_scan(x, oracle.dv_segments(N30, 8), "plus"))


def _config_tests(*argv, timeout=600):
    import json
    import os
    import subprocess
    exe = os.path.join(os.path.dirname(os.path.abspath(__file__)), "cpp", "bin", "config_tests")
    r = subprocess.run([exe, *argv], capture_output=True, text=True, timeout=timeout)
    print(r.stdout[-3000:], r.stderr[-2000:])
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert line, r.stdout[-2000:] + r.stderr[-2000:]
    return json.loads(line[-1]), r.returncode


@pytest.mark.parametrize("dtype", ["f32", "i32"])
def test_c2_cpp_dropin_2pow30_eight_segments(dtype):
    """C2 through the C++ drop-in at config size, the reference's call
    sequence (test/gtest/shp/shp-tests.cpp:34-39, algorithms.cpp:61-149):
    shp::reduce(par_unseq, dv, 0) then shp::inclusive_scan(par_unseq, dv,
    out) on distributed_vector<float|int32_t>(2^30) over 8 segments
    duplicated on one GPU.  The pieces sit on distinct segments, so the scan
    runs the pinned-totals tile path (drhip_reduce_tiles per piece, totals
    folded on the device; include/dr/shp/algorithms.hpp inclusive_scan_impl).
    f32: reduce rel <= 1e-5, every element rel <= 1e-5 vs the fp64 prefix;
    i32: bit-exact vs orc_shp_reduce_i32 / orc_shp_scan_i32 over the same
    pieces.  Two calls (cold and warm workspaces), both checked."""
    res, rc = _config_tests("c2", "30", "8", "--dtype", dtype)
    assert res["elements"] == N30 and res["segments"] == 8 and res["pieces"] == 8
    assert res["path"] == "tiles_pinned_totals"
    assert res["segment_sizes"] == [1 << 27] * 8 and res["size_mismatches"] == 0
    assert res["scan_mismatches"] == [0, 0]
    if dtype == "f32":
        assert res["reduce_rel_err"] <= FP_RTOL and max(res["scan_max_rel_err"]) <= FP_RTOL
    else:
        assert res["reduce_exact"]
    assert res["ok"] and rc == 0


@pytest.mark.parametrize("dtype", ["f32", "i32"])
def test_c2_cpp_dropin_misaligned_2pow27(dtype):
    """The same sequence with an output of n + 8*1001 elements: its segment
    boundaries fall inside the input's, so consecutive zipped pieces share an
    input segment (15 pieces) and inclusive_scan takes the host-fold path
    (piece totals by drhip_reduce, carries folded on the host, single-pass
    scans with carry-in)."""
    res, rc = _config_tests("c2", "27", "8", "--dtype", dtype, "--misaligned", "1001")
    assert res["elements"] == 1 << 27 and res["out_elements"] == (1 << 27) + 8 * 1001
    assert res["path"] == "host_fold" and res["pieces"] == 15
    assert res["scan_mismatches"] == [0, 0]
    if dtype == "f32":
        assert res["reduce_rel_err"] <= FP_RTOL and max(res["scan_max_rel_err"]) <= FP_RTOL
    else:
        assert res["reduce_exact"]
    assert res["ok"] and rc == 0


# ------------------------------------------------------------------ C3

def test_c3_sort_u32_2pow28(dr, oracle):
    n = 1 << 28
    x = np.random.default_rng(1).integers(0, 1 << 32, n, dtype=np.uint32)
    buf = dr.DeviceArray(0, n, np.uint32, host=x)
    ws = dr.sort_workspace(0, np.uint32, n)
    tmp = dr.DeviceArray(0, ws, np.uint8)
    try:
        dr.sort_async(0, np.uint32, buf.ptr, n, tmp.ptr, ws)
        got = buf.numpy()
    finally:
        buf.free()
        tmp.free()
    assert np.array_equal(got, oracle.sort_u32_large(x))


def test_c3_sort_u32_2pow31_eight_segments_distributed():
    """C3 at its CONFIGURED global size in its distributed form: shp::sort
    (C++ drop-in, include/dr/shp/sort.hpp) of a distributed_vector<uint32_t>
    of 2^31 keys over 8 segments duplicated on one GPU (the reference's
    --devicesCount method, test/gtest/shp/shp-tests.cpp:34-39): 8 local
    radix sorts of 2^28, exact splitting, 64 piece copies, drhip_merge_runs
    of 8 runs per destination (2^28 keys each), copy back.  tests/cpp/bin/
    config_tests checks every key bit-exact against the oracle's radix sort
    (orc_radix_sort_u32_par, pinned to the qsort restatement) and every
    segment size against ceil(n/P) (shp/distributed_vector.hpp:142)."""
    import json
    import os
    import subprocess
    exe = os.path.join(os.path.dirname(os.path.abspath(__file__)), "cpp", "bin", "config_tests")
    r = subprocess.run([exe, "31", "8", "--threads", "16"], capture_output=True, text=True, timeout=600)
    print(r.stdout[-3000:], r.stderr[-2000:])
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert line, r.stdout[-2000:] + r.stderr[-2000:]
    res = json.loads(line[-1])
    assert res["keys"] == 1 << 31 and res["segments"] == 8
    assert res["segment_sizes"] == [1 << 28] * 8
    assert res["size_mismatches"] == 0 and res["key_mismatches"] == 0
    assert res["ok"] and r.returncode == 0


@pytest.mark.parametrize("log2n,segments", [(28, 1), (31, 8)])
def test_c3_sort_greater_u32(log2n, segments):
    """shp::sort(par_unseq, dv, std::greater<>()) (SURVEY.md 8a A10:
    std::ranges::sort semantics with a comparator): the keys flipped by an
    order-reversing bit inversion, sorted ascending, flipped back.  Every key
    bit-exact against the oracle's radix sort reversed, on one segment of
    2^28 and in C3's distributed form (2^31 over 8 segments)."""
    res, rc = _config_tests(str(log2n), str(segments), "--greater", "--threads", "16")
    assert res["order"] == "greater" and res["keys"] == 1 << log2n and res["segments"] == segments
    assert res["size_mismatches"] == 0 and res["key_mismatches"] == 0
    assert res["ok"] and rc == 0


@pytest.mark.parametrize("order", ["less", "greater"])
def test_c3_sort_lambda_u32_2pow31_eight_segments(order):
    """C3 at its configured size through the GENERAL-comparator tier:
    shp::sort(par_unseq, dv, [](a, b) { return a < b; }) (or a > b) on
    2^31 keys over 8 segments -- a lambda the drop-in cannot identify as
    std::less / std::greater, so it runs the stable merge sort of
    dr/shp/merge_sort.hpp (8 local sorts, comparator-based exact splitting,
    pairwise run merges).  Every key bit-exact against the oracle's sort."""
    extra = ["--greater"] if order == "greater" else []
    res, rc = _config_tests("31", "8", "--lambda", *extra, "--threads", "16")
    assert res["comparator"].startswith("lambda") and res["order"] == order
    assert res["keys"] == 1 << 31 and res["segments"] == 8 and res["segment_sizes"] == [1 << 28] * 8
    assert res["size_mismatches"] == 0 and res["key_mismatches"] == 0
    assert res["ok"] and rc == 0


# ------------------------------------------------------------------ C4

def _c4_windows(m, rng, width=1024, count=48):
    starts = {0, m - width}
    for k in range(1, 8):  # the 8-way row-tile edges
        starts.add(k * m // 8 - width // 2)
    starts.update(int(s) for s in rng.integers(0, m - width, count))
    return sorted(starts)


@pytest.mark.parametrize("kind", ["banded", "random"])
def test_c4_gemv_2pow26(dr, oracle, kind):
    m = 1 << 26
    k = 10
    kc = 0 if kind == "banded" else 1
    nnz = dr.csr_nnz(kc, 0, m, m, k)
    x = np.random.default_rng(5).random(m, dtype=np.float32)
    rp = dr.DeviceArray(0, m + 1, np.int32)
    ci = dr.DeviceArray(0, nnz, np.int32)
    va = dr.DeviceArray(0, nnz, np.float32)
    xd = dr.DeviceArray(0, m, np.float32, host=x)
    y = dr.DeviceArray(0, m, np.float32, host=np.zeros(m, np.float32))
    try:
        dr.csr_gen(0, kc, 0, m, m, k, 1, rp.ptr, ci.ptr, va.ptr)
        dr.spmv_csr(0, m, nnz, rp.ptr, ci.ptr, va.ptr, xd.ptr, y.ptr)
        got = y.numpy()
    finally:
        for b in (rp, ci, va, xd, y):
            b.free()
    for s in _c4_windows(m, np.random.default_rng(9)):
        orp, oci, ova = oracle.csr_gen(kind, s, 1024, m, 1, k=k)
        ref = oracle.csr_spmv(orp, oci, ova, x, np.zeros(1024, np.float32))
        err = np.max(np.abs(got[s:s + 1024] - ref) / np.maximum(np.abs(ref), 1e-30))
        assert err <= FP_RTOL, (kind, s, err)


@pytest.mark.parametrize("kind", ["banded", "random"])
def test_c4_gemv_row_tile(dr, oracle, kind):
    """One of the 8 row tiles of C4 (rows [3m/8, 4m/8), tile-local rowptr,
    global columns), every row of the tile vs the oracle."""
    m = 1 << 26
    row0, rows, k = 3 * m // 8, m // 8, 10
    kc = 0 if kind == "banded" else 1
    nnz = dr.csr_nnz(kc, row0, rows, m, k)
    x = np.random.default_rng(6).random(m, dtype=np.float32)
    rp = dr.DeviceArray(0, rows + 1, np.int32)
    ci = dr.DeviceArray(0, nnz, np.int32)
    va = dr.DeviceArray(0, nnz, np.float32)
    xd = dr.DeviceArray(0, m, np.float32, host=x)
    y0 = np.random.default_rng(7).random(rows, dtype=np.float32)
    y = dr.DeviceArray(0, rows, np.float32, host=y0)
    try:
        dr.csr_gen(0, kc, row0, rows, m, k, 1, rp.ptr, ci.ptr, va.ptr)
        dr.spmv_csr(0, rows, nnz, rp.ptr, ci.ptr, va.ptr, xd.ptr, y.ptr)
        got = y.numpy()
    finally:
        for b in (rp, ci, va, xd, y):
            b.free()
    orp, oci, ova = oracle.csr_gen(kind, row0, rows, m, 1, k=k)
    ref = oracle.csr_spmv(orp, oci, ova, x, y0)  # c += A*b (accumulates)
    assert max_rel_err(got, ref) <= FP_RTOL


@pytest.mark.parametrize("kind,index", [("banded", "i64"), ("random", "i64"), ("banded", "i32")])
def test_c4_cpp_dropin_gemv_2pow26_eight_segments(kind, index):
    """C4 through the C++ drop-in at config size: shp::gemv(c, a, b) on a
    shp::sparse_matrix<float> of 2^26 x 2^26 with the reference's default
    index type I = std::size_t (containers/sparse_matrix.hpp:126), 8 {8, 1}
    row tiles duplicated on one GPU, b and c distributed_vector<float>
    (algorithms/gemv.hpp:13-71, intended c += A*b): every tile's window of b
    gathered by device-to-device copies of b's segments, then the tile SpMV.
    Two gemv calls accumulate (c = 2 A b).  tests/cpp/bin/config_tests checks
    4096-row windows at both ends, every tile edge and 64 random places, each
    row rel <= 1e-5 vs the oracle's generator + fp64 CSR rows."""
    res, rc = _config_tests("c4", "26", "8", "--kind", kind, "--index", index)
    assert res["rows"] == 1 << 26 and res["segments"] == 8 and res["kind"] == kind
    assert res["index_bytes"] == (8 if index == "i64" else 4)
    assert res["rows_checked"] >= 4096 * (2 + 7 + 64) and res["row_mismatches"] == 0
    assert res["max_rel_err"] <= FP_RTOL
    assert res["ok"] and rc == 0


# ------------------------------------------------------------------ C5

def test_c5_stencil1d_2pow29(dr, oracle):
    n = 1 << 29
    x = np.random.default_rng(3).random(n + 2, dtype=np.float32)
    src = dr.DeviceArray(0, n + 2, np.float32, host=x)
    dst = dr.DeviceArray(0, n + 2, np.float32, host=np.zeros(n + 2, np.float32))
    try:
        dr.stencil1d(0, np.float32, src.ptr, dst.ptr, n, 1, 0, n)
        got = dst.numpy()
    finally:
        src.free()
        dst.free()
    assert np.array_equal(got, oracle.stencil1d(x, 1, out=np.zeros(n + 2, np.float32)))


def test_c5_stencil2d_8192x65536(dr, oracle):
    nx, rows = 65536, 8192
    x = np.random.default_rng(4).random((rows + 2) * nx, dtype=np.float32)
    src = dr.DeviceArray(0, x.size, np.float32, host=x)
    dst = dr.DeviceArray(0, x.size, np.float32, host=x)
    try:
        dr.stencil2d(0, np.float32, src.ptr, dst.ptr, nx, rows, 0, rows)
        got = dst.numpy()
    finally:
        src.free()
        dst.free()
    assert np.array_equal(got, oracle.stencil2d(x, nx, rows + 2, out=x.copy()))


def test_c5_stencil1d_eight_segments_halo(dr, oracle):
    """8 segments x 2^26 int32 cells (the C5 row-block layout of 8 GPUs, one
    GPU's worth per segment), span_halo exchange of one cell per side by
    device-to-device copies between steps, 3 steps, global ends fixed
    (examples/mhp/stencil-1d.cpp).  Every cell bit-exact vs the oracle run
    on the undistributed array."""
    P, seg, steps = 8, 1 << 26, 3
    n = P * seg
    a = np.random.default_rng(8).integers(-1000, 1000, n, dtype=np.int32)
    dr.finalize()
    dr.init([0] * P)
    bufs = []
    try:
        for which in (a, a):
            row = []
            for r in range(P):
                host = np.zeros(seg + 2, np.int32)
                host[1:seg + 1] = which[r * seg:(r + 1) * seg]
                row.append(dr.DeviceArray(r, seg + 2, np.int32, host=host))
            bufs.append(row)
        cur = 0
        for _ in range(steps):
            src, dstb = bufs[cur], bufs[cur ^ 1]
            for r in range(P):  # halo.hpp:358-386 owned/halo groups, radius 1
                if r > 0:
                    dr.d2d(r, src[r - 1].at(seg + 1), src[r].at(1), 4)
                if r + 1 < P:
                    dr.d2d(r, src[r + 1].at(0), src[r].at(seg), 4)
            dr.sync()
            for r in range(P):
                lo, hi = (1 if r == 0 else 0), (seg - 1 if r == P - 1 else seg)
                dr.stencil1d(r, np.int32, src[r].ptr, dstb[r].ptr, seg, 1, lo, hi)
            dr.sync()
            cur ^= 1
        got = np.concatenate([bufs[cur][r].numpy()[1:seg + 1] for r in range(P)])
    finally:
        for row in bufs:
            for b in row:
                b.free()
        dr.finalize()
        dr.init([0])
    ref = a.copy()
    for _ in range(steps):
        ref = oracle.stencil1d(ref, 1, out=ref.copy())  # interior updated, ends fixed
    assert np.array_equal(got, ref)


def test_c5_stencil1d_2pow32_eight_segments_halo(dr, oracle):
    """C5 at its CONFIGURED global size: 2^32 fp32 cells as 8 segments of
    2^29 (one GPU's share each, duplicated on one GPU), radius-1 span_halo
    exchange by device-to-device copies before every step (halo.hpp:358-386),
    3 steps of the 3-point stencil (examples/mhp/stencil-1d.cpp:16-19), global
    ends fixed.  After 3 steps a cell depends on the 7 initial cells around
    it, so every segment edge (+-4096 cells around each of the 7 internal
    boundaries and the two global ends) and 64 random interior windows of
    4096 cells are checked bit-exact against the oracle's stencil run 3
    steps on the initial values around the window (the same left-to-right
    fp32 order: (p[-1] + p[0]) + p[1])."""
    import torch
    P, seg, steps, W = 8, 1 << 29, 3, 4096
    n = P * seg
    dr.finalize()
    dr.init([0] * P)
    try:
        g = torch.Generator(device="cuda").manual_seed(55)
        bufs = [[torch.empty(seg + 2, dtype=torch.float32, device="cuda") for _ in range(P)] for _ in range(2)]
        for r in range(P):
            bufs[0][r][1:seg + 1].copy_(torch.rand(seg, generator=g, device="cuda"))
            bufs[0][r][0] = 0.0
            bufs[0][r][seg + 1] = 0.0
            bufs[1][r].copy_(bufs[0][r])
        rng = np.random.default_rng(5)
        starts = {0, n - W}
        for k in range(1, P):
            starts.add(k * seg - W)
            starts.add(k * seg)
        starts.update(int(v) for v in rng.integers(steps, n - W - steps, 64))
        starts = sorted(starts)

        def window(bset, a, b):  # global cells [a, b) of one buffer set, on the host
            out = []
            while a < b:
                r, o = divmod(a, seg)
                take = min(b - a, seg - o)
                out.append(bset[r][1 + o:1 + o + take].cpu().numpy())
                a += take
            return np.concatenate(out)

        init = {s0: window(bufs[0], max(0, s0 - steps), min(n, s0 + W + steps)) for s0 in starts}
        torch.cuda.synchronize()
        cur = 0
        for _ in range(steps):
            src, dstb = bufs[cur], bufs[cur ^ 1]
            for r in range(P):  # radius-1 owned/halo groups
                if r > 0:
                    dr.d2d(r, src[r - 1].data_ptr() + 4 * (seg + 1), src[r].data_ptr() + 4, 4)
                if r + 1 < P:
                    dr.d2d(r, src[r + 1].data_ptr(), src[r].data_ptr() + 4 * seg, 4)
            dr.sync()
            for r in range(P):
                lo, hi = (1 if r == 0 else 0), (seg - 1 if r == P - 1 else seg)
                dr.stencil1d(r, np.float32, src[r].data_ptr(), dstb[r].data_ptr(), seg, 1, lo, hi)
            dr.sync()
            cur ^= 1
        bad = 0
        for s0 in starts:
            a = max(0, s0 - steps)
            ref = init[s0].copy()
            for _ in range(steps):
                ref = oracle.stencil1d(ref, 1, out=ref.copy())
            # the window's own cells; the oracle's artificial ends at a and
            # b only disturb cells within `steps` of them, unless they are
            # the global ends (fixed in both)
            got = window(bufs[cur], s0, s0 + W)
            bad += int(np.count_nonzero(got != ref[s0 - a:s0 - a + W]))
        del bufs
        torch.cuda.empty_cache()
    finally:
        dr.finalize()
        dr.init([0])
    assert bad == 0, f"{bad} cells differ"


def test_c5_stencil2d_2pow16_square_eight_row_blocks_halo(dr, oracle):
    """C5's 2-D form at its CONFIGURED size: a 2^16 x 2^16 fp32 grid as 8
    row-block segments of 8192 x 65536 (one GPU's share each, duplicated on
    one GPU), each stored as [halo row | 8192 owned rows | halo row].  Before
    every step the span_halo exchange with a ROW as the cell
    (details/halo.hpp:358-386: the first owned row to rank-1's lower halo,
    the last owned row to rank+1's upper halo) runs as device-to-device
    copies; then 3 steps of drhip_stencil2d (5-point, c + w + e + n + s),
    global edge rows and columns fixed.  After 3 steps a cell depends on the
    initial cells within 3 rows/columns, so every segment-boundary band
    (+-8 rows around each of the 7 internal boundaries), both global edge
    bands and 64 random interior windows of 8 full rows are checked
    bit-exact against oracle.stencil2d run 3 steps on the initial rows
    around the window."""
    import torch
    P, rows, nx, steps = 8, 8192, 1 << 16, 3
    ny = P * rows
    H = 8  # rows per checked window
    dr.finalize()
    dr.init([0] * P)
    try:
        g = torch.Generator(device="cuda").manual_seed(66)
        bufs = [[torch.empty((rows + 2) * nx, dtype=torch.float32, device="cuda") for _ in range(P)]
                for _ in range(2)]
        for r in range(P):
            v = bufs[0][r].view(rows + 2, nx)
            v[1:rows + 1].copy_(torch.rand(rows, nx, generator=g, device="cuda"))
            v[0].zero_()
            v[rows + 1].zero_()
            bufs[1][r].copy_(bufs[0][r])  # fixed edge columns / global rows
        rng = np.random.default_rng(6)
        starts = {0, ny - H}
        for k in range(1, P):
            starts.add(k * rows - H)
            starts.add(k * rows)
        starts.update(int(v) for v in rng.integers(steps, ny - H - steps, 64))
        starts = sorted(starts)

        def band(bset, a, b):  # global rows [a, b) of one buffer set, on the host
            out = []
            while a < b:
                r, o = divmod(a, rows)
                take = min(b - a, rows - o)
                out.append(bset[r].view(rows + 2, nx)[1 + o:1 + o + take].cpu().numpy())
                a += take
            return np.concatenate(out)

        init = {s0: band(bufs[0], max(0, s0 - steps), min(ny, s0 + H + steps)) for s0 in starts}
        torch.cuda.synchronize()
        rb = nx * 4  # one row, in bytes
        cur = 0
        for _ in range(steps):
            src, dstb = bufs[cur], bufs[cur ^ 1]
            for r in range(P):  # radius-1 owned/halo groups, a row per cell
                if r > 0:  # rank r-1's last owned row -> my upper halo (row 0)
                    dr.d2d(r, src[r].data_ptr(), src[r - 1].data_ptr() + rows * rb, rb)
                if r + 1 < P:  # rank r+1's first owned row -> my lower halo (row rows+1)
                    dr.d2d(r, src[r].data_ptr() + (rows + 1) * rb, src[r + 1].data_ptr() + rb, rb)
            dr.sync()
            for r in range(P):
                rlo, rhi = (1 if r == 0 else 0), (rows - 1 if r == P - 1 else rows)
                dr.stencil2d(r, np.float32, src[r].data_ptr(), dstb[r].data_ptr(), nx, rows, rlo, rhi)
            dr.sync()
            cur ^= 1
        bad = 0
        for s0 in starts:
            a = max(0, s0 - steps)
            ref = init[s0].reshape(-1)
            sub = ref.size // nx
            for _ in range(steps):
                ref = oracle.stencil2d(ref, nx, sub, out=ref.copy())
            got = band(bufs[cur], s0, s0 + H)
            bad += int(np.count_nonzero(got.reshape(-1) != ref[(s0 - a) * nx:(s0 - a + H) * nx]))
        del bufs
        torch.cuda.empty_cache()
    finally:
        dr.finalize()
        dr.init([0])
    assert bad == 0, f"{bad} cells differ"
