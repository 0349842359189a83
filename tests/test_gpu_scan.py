"""GPU parity: drhip_inclusive_scan (C-ABI, single-pass decoupled look-back)
against the oracle's restatement of shp::inclusive_scan.

Integers: bit-exact, including wrapping products.  Floats: per-element
relative error <= 1e-5 against the fp64 sequential prefix (SURVEY.md 8d:
a sequential fp32 scan is not a usable oracle at these sizes)."""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

FP_RTOL = 1e-5
GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "shp_known_answers.json")


def ref_scan(oracle, x, op, init=None, carry=None):
    if x.dtype.kind == "f":
        r = oracle.scan_exact_f32(x.astype(np.float32) if x.dtype == np.float32 else x, op, init)
        if x.dtype == np.float64:
            r = np.empty(x.size)
            acc = None
            for i, v in enumerate(x):  # small sizes only
                acc = (v if init is None else _op(op, init, v)) if i == 0 else _op(op, acc, v)
                r[i] = acc
        if carry is not None:
            r = _op(op, r, carry)
        return r
    out = oracle.shp_scan(x, [x.size], op, init)
    if carry is not None:
        c = np.array([carry], dtype=x.dtype)
        out = oracle.shp_scan(np.concatenate([c, x]), [x.size + 1], op, None)[1:]
        if init is not None:
            out = oracle.shp_scan(np.concatenate([c, np.array([init], x.dtype), x]), [x.size + 2], op)[2:]
    return out


def _op(op, a, b):
    return {"plus": np.add, "mul": np.multiply, "min": np.minimum, "max": np.maximum}[op](a, b)


def check(got, ref, dtype):
    if np.dtype(dtype).kind == "f":
        denom = np.maximum(np.abs(ref), 1e-30)
        err = np.max(np.abs(got.astype(np.float64) - ref) / denom) if ref.size else 0
        assert err <= FP_RTOL, err
    else:
        assert np.array_equal(got, ref.astype(dtype)), np.nonzero(got != ref)[0][:10]


def make_input(dtype, op, n, seed):
    rng = np.random.default_rng(seed)
    dt = np.dtype(dtype)
    if dt.kind == "f":
        if op == "mul":
            return (1.0 + (rng.random(n) - 0.5) * 1e-4).astype(dt)
        if op in ("min", "max"):
            return (rng.random(n) - 0.5).astype(dt)
        return rng.random(n).astype(dt)
    info = np.iinfo(dt)
    if op == "mul":
        return rng.integers(1, 1 << 20, size=n, dtype=np.int64).astype(dt) | 1
    return rng.integers(info.min, info.max, size=n, endpoint=True, dtype=dt)


SIZES = [1, 5, 4095, 4096, 4097, 2048 * 3 + 1, 100000, (1 << 21) + 5]


@pytest.mark.parametrize("dtype", [np.int32, np.uint32, np.int64, np.uint64, np.float32])
@pytest.mark.parametrize("op", ["plus", "mul", "min", "max"])
@pytest.mark.parametrize("n", SIZES)
def test_scan_parity(dr, oracle, dtype, op, n):
    x = make_input(dtype, op, n, seed=n + len(op))
    src = dr.DeviceArray(0, n, dtype, host=x)
    dst = dr.DeviceArray(0, n, dtype)
    dr.scan_async(0, dtype, op, src.ptr, dst.ptr, n)
    check(dst.numpy(), ref_scan(oracle, x, op), dtype)
    src.free()
    dst.free()


@pytest.mark.parametrize("dtype", [np.int32, np.float32, np.int64])
@pytest.mark.parametrize("n,in_off,out_off", [(1000, 1, 0), (9001, 0, 3), (50000, 2, 1), (4096, 1, 1)])
def test_scan_misaligned(dr, oracle, dtype, n, in_off, out_off):
    """Sub-range pointers (zipped pieces of misaligned segments) take the
    scalar path; results must be identical."""
    x = make_input(dtype, "plus", n + in_off, seed=n)
    src = dr.DeviceArray(0, n + in_off, dtype, host=x)
    dst = dr.DeviceArray(0, n + out_off, dtype)
    dr.scan_async(0, dtype, "plus", src.at(in_off), dst.at(out_off), n)
    check(dst.numpy()[out_off:], ref_scan(oracle, x[in_off:], "plus"), dtype)
    src.free()
    dst.free()


@pytest.mark.parametrize("dtype", [np.int32, np.float32])
@pytest.mark.parametrize("n", [3, 4097, 123457])
def test_scan_inplace_init_carry_total(dr, oracle, dtype, n):
    x = make_input(dtype, "plus", n, seed=5)
    buf = dr.DeviceArray(0, n, dtype, host=x)
    acc = np.float64 if np.dtype(dtype).kind == "f" else dtype
    tot = dr.DeviceArray(0, 1, acc)
    init = dtype(12) if np.dtype(dtype).kind != "f" else dtype(0.5)
    carry = acc(-7) if np.dtype(dtype).kind != "f" else acc(3.25)
    dr.scan_async(0, dtype, "plus", buf.ptr, buf.ptr, n, init=init, carry=carry, total_dev=tot.ptr)
    got = buf.numpy()
    if np.dtype(dtype).kind == "f":
        ref = np.cumsum(x.astype(np.float64)) + float(init) + float(carry)
        check(got, ref, dtype)
        assert abs(tot.numpy()[0] - ref[-1]) <= FP_RTOL * ref[-1]  # fp32 in-tile sums
    else:
        ref = ref_scan(oracle, x, "plus", init=init, carry=carry)
        check(got, ref, dtype)
        assert tot.numpy()[0] == ref[-1]
    buf.free()
    tot.free()


def test_scan_carry_from_device(dr, oracle):
    """carry_dev: the carry is read by the kernel (e.g. an RCCL result)."""
    n = 77777
    x = make_input(np.int32, "plus", n, seed=9)
    src = dr.DeviceArray(0, n, np.int32, host=x)
    dst = dr.DeviceArray(0, n, np.int32)
    c = dr.DeviceArray(0, 1, np.int32, host=np.array([1000003], dtype=np.int32))
    dr.scan_async(0, np.int32, "plus", src.ptr, dst.ptr, n, carry_dev=c.ptr)
    check(dst.numpy(), ref_scan(oracle, x, "plus", carry=np.int32(1000003)), np.int32)
    for b in (src, dst, c):
        b.free()


@pytest.mark.parametrize("dtype,op", [(np.int32, "plus"), (np.float32, "plus"), (np.int64, "max"),
                                      (np.float64, "plus"), (np.uint32, "mul")])
@pytest.mark.parametrize("w,rank", [(1, 0), (2, 1), (8, 0), (8, 5), (8, 7)])
def test_scan_gathered_equals_fold_then_carry(dr, dtype, op, w, rank):
    """drhip_inclusive_scan_gathered (the scan kernel folds the gathered
    segment partials itself) equals the two-kernel form it replaces:
    drhip_fold_partials -> carry + result, then the scan reading the carry
    from device memory -- bit-identical results and integer scans; float
    scans to rounding (the look-back's grouping varies run to run)."""
    n = 300001
    x = make_input(dtype, op, n, seed=11 + w + rank)
    acc = dr.ACC_OF[dr.DTYPES[np.dtype(dtype)]]
    parts = np.random.default_rng(w * 10 + rank).integers(1, 50, w).astype(acc)
    if np.dtype(acc).kind == "f":
        parts = parts * np.float64(1.000001)
    src = dr.DeviceArray(0, n, dtype, host=x)
    d1, d2 = dr.DeviceArray(0, n, dtype), dr.DeviceArray(0, n, dtype)
    g = dr.DeviceArray(0, w, acc, host=parts)
    res1, res2 = dr.DeviceArray(0, 1, acc), dr.DeviceArray(0, 1, acc)
    car = dr.DeviceArray(0, 1, acc)
    try:
        dr.fold_partials_async(0, acc, op, g.ptr, w, rank, res1.ptr, car.ptr if rank else None)
        dr.scan_async(0, dtype, op, src.ptr, d1.ptr, n, carry_dev=car.ptr if rank else None)
        dr.scan_gathered_async(0, dtype, op, src.ptr, d2.ptr, n, g.ptr, w, rank, res2.ptr)
        a, b = d1.numpy(), d2.numpy()
        if np.dtype(dtype).kind == "f":
            # the look-back folds predecessors' aggregates in a timing-dependent
            # grouping: float scans agree to rounding, not bit for bit
            ref = a.astype(np.float64)
            assert np.max(np.abs(b - ref) / np.maximum(np.abs(ref), 1e-300)) <= (1e-5 if dtype == np.float32 else 1e-12)
        else:
            assert np.array_equal(a.view(np.uint8), b.view(np.uint8))
        assert np.array_equal(res1.numpy().view(np.uint8), res2.numpy().view(np.uint8))
    finally:
        for buf in (src, d1, d2, g, res1, res2, car):
            buf.free()


TILE_SIZES = [1, 1000, 65537, (1 << 20) + 37, (1 << 25) + 5]  # the last one at the big-tile shape


@pytest.mark.parametrize("dtype,op", [(np.int32, "plus"), (np.float32, "plus"), (np.int64, "plus"),
                                      (np.uint32, "max"), (np.float64, "min"), (np.int32, "mul")])
@pytest.mark.parametrize("n", TILE_SIZES)
@pytest.mark.parametrize("shift", [0, 1])
def test_reduce_tiles_then_scan_tiles(dr, oracle, dtype, op, n, shift):
    """drhip_reduce_tiles + drhip_inclusive_scan_tiles (the reduce's tile
    prefixes replace the scan's look-back): the reduce equals the oracle's
    (bit-exact for integers), every scanned element equals the oracle scan
    (bit-exact for integers, rel <= 1e-5 for floats), at both tile shapes and
    on ranges that start off a 16-byte boundary."""
    if np.dtype(dtype) == np.float64 and n > 70000:
        pytest.skip("fp64 reference scan is a Python loop")
    x = make_input(dtype, op, n + shift, seed=n % 97 + shift)
    acc = dr.ACC_OF[dr.DTYPES[np.dtype(dtype)]]
    src = dr.DeviceArray(0, n + shift, dtype, host=x)
    dst = dr.DeviceArray(0, n + shift, dtype)
    red = dr.DeviceArray(0, 1, acc)
    try:
        dr.reduce_tiles_async(0, dtype, op, src.at(shift), n, red.ptr)
        dr.scan_tiles_async(0, dtype, op, src.at(shift), dst.at(shift), n)
        got, got_r = dst.numpy()[shift:], red.numpy()[0]
    finally:
        for b in (src, dst, red):
            b.free()
    xs = x[shift:]
    check(got, ref_scan(oracle, xs, op), dtype)
    if np.dtype(dtype).kind == "f":
        ref_r = float(ref_scan(oracle, xs, op)[-1]) if op != "plus" else oracle.reduce_exact(xs)
        assert abs(float(got_r) - ref_r) <= 1e-5 * max(abs(ref_r), 1e-30)
    else:
        assert np.array_equal(np.array([got_r]).astype(dtype), ref_scan(oracle, xs, op)[-1:].astype(dtype))


@pytest.mark.parametrize("dtype", [np.int32, np.float32])
@pytest.mark.parametrize("w,rank", [(1, 0), (8, 0), (8, 5)])
def test_scan_tiles_carries(dr, dtype, w, rank):
    """The tile scan with a device carry and with gathered partials folds
    them exactly as drhip_inclusive_scan_gathered / carry_dev do: bit-identical
    to fold_partials + the single-pass scan for integers, within 1e-5 for
    fp32 (different tile-prefix summation order)."""
    n = (1 << 22) + 999
    x = make_input(dtype, "plus", n, seed=3 + rank)
    acc = dr.ACC_OF[dr.DTYPES[np.dtype(dtype)]]
    parts = (np.arange(w) * 7 + 3).astype(acc)
    src = dr.DeviceArray(0, n, dtype, host=x)
    d1, d2, d3 = (dr.DeviceArray(0, n, dtype) for _ in range(3))
    g = dr.DeviceArray(0, w, acc, host=parts)
    r1, r2, car, red = (dr.DeviceArray(0, 1, acc) for _ in range(4))
    try:
        dr.fold_partials_async(0, acc, "plus", g.ptr, w, rank, r1.ptr, car.ptr if rank else None)
        dr.scan_async(0, dtype, "plus", src.ptr, d1.ptr, n, carry_dev=car.ptr if rank else None)
        dr.reduce_tiles_async(0, dtype, "plus", src.ptr, n, red.ptr)
        dr.scan_tiles_async(0, dtype, "plus", src.ptr, d2.ptr, n, partials=g.ptr, w=w, rank=rank, result=r2.ptr)
        dr.scan_tiles_async(0, dtype, "plus", src.ptr, d3.ptr, n, carry_dev=car.ptr if rank else None)
        a, b, c = d1.numpy(), d2.numpy(), d3.numpy()
        assert np.array_equal(r1.numpy(), r2.numpy())
    finally:
        for buf in (src, d1, d2, d3, g, r1, r2, car, red):
            buf.free()
    if np.dtype(dtype).kind == "i":
        assert np.array_equal(a, b) and np.array_equal(a, c)
    else:
        ref = a.astype(np.float64)
        assert np.max(np.abs(b - ref) / np.abs(ref)) <= 1e-5 and np.max(np.abs(c - ref) / np.abs(ref)) <= 1e-5


def test_scan_tiles_refuses_another_range(dr):
    """The tile prefixes describe ONE range: scanning any other (pointer,
    size, dtype or op) is refused, not computed from stale prefixes."""
    n = 100000
    x = make_input(np.int32, "plus", n, seed=1)
    src = dr.DeviceArray(0, n, np.int32, host=x)
    dst = dr.DeviceArray(0, n, np.int32)
    red = dr.DeviceArray(0, 1, np.int32)
    try:
        dr.reduce_tiles_async(0, np.int32, "plus", src.ptr, n, red.ptr)
        for args in ((src.at(1), n - 1, np.int32, "plus"), (src.ptr, n - 1, np.int32, "plus"),
                     (src.ptr, n, np.uint32, "plus"), (src.ptr, n, np.int32, "max")):
            with pytest.raises(dr.DrhipError):
                dr.scan_tiles_async(0, args[2], args[3], args[0], dst.ptr, args[1])
        dr.scan_tiles_async(0, np.int32, "plus", src.ptr, dst.ptr, n)
        assert np.array_equal(dst.numpy(), np.cumsum(x.astype(np.int64)).astype(np.int32))
    finally:
        for b in (src, dst, red):
            b.free()


def test_scan_tiles_inplace_and_counter_resets(dr):
    """In-place tile scan (the persistent pipeline loads tile t+1 before it
    stores tile t, never the same tile), then back-to-back reduce + scan
    pairs of different sizes (grids of different widths): the self-resetting
    tile counters must start every launch at tile 0 -- a stale counter would
    skip tiles and leave them unscanned."""
    for n in [(1 << 21) + 3, 5000, 3, (1 << 20), 1, (1 << 22) + 17]:
        x = make_input(np.int32, "plus", n, seed=n % 101)
        buf = dr.DeviceArray(0, n, np.int32, host=x)
        red = dr.DeviceArray(0, 1, np.int32)
        try:
            dr.reduce_tiles_async(0, np.int32, "plus", buf.ptr, n, red.ptr)
            dr.scan_tiles_async(0, np.int32, "plus", buf.ptr, buf.ptr, n)
            got, got_r = buf.numpy(), red.numpy()[0]
        finally:
            buf.free()
            red.free()
        ref = np.cumsum(x.astype(np.int64)).astype(np.int32)
        assert np.array_equal(got, ref), (n, np.nonzero(got != ref)[0][:5])
        assert got_r == ref[-1]


@pytest.mark.parametrize("kind", ["tiles", "gathered"])
@pytest.mark.parametrize("dtype,op", [(np.int32, "plus"), (np.float32, "plus"), (np.int64, "max")])
def test_scan_empty_segment_still_writes_result(dr, dtype, op, kind):
    """With the ceil(n/N) split trailing ranks can own empty segments (n = 9,
    N = 8: ranks 5-7 hold nothing).  Their scan of n == 0 still delivers the
    fold of all w gathered partials in *result (drhip_fold_partials' order),
    never a stale value."""
    w = 8
    acc = dr.ACC_OF[dr.DTYPES[np.dtype(dtype)]]
    parts = (np.arange(w) * 5 + 2).astype(acc)
    g = dr.DeviceArray(0, w, acc, host=parts)
    ref, res = dr.DeviceArray(0, 1, acc), dr.DeviceArray(0, 1, acc, host=np.full(1, 77, acc))
    buf = dr.DeviceArray(0, 16, dtype)
    red = dr.DeviceArray(0, 1, acc)
    try:
        dr.fold_partials_async(0, acc, op, g.ptr, w, 6, ref.ptr, None)
        if kind == "tiles":
            dr.reduce_tiles_async(0, dtype, op, buf.ptr, 0, red.ptr)
            dr.scan_tiles_async(0, dtype, op, buf.ptr, buf.ptr, 0, partials=g.ptr, w=w, rank=6, result=res.ptr)
        else:
            dr.scan_gathered_async(0, dtype, op, buf.ptr, buf.ptr, 0, g.ptr, w, 6, res.ptr)
        got, want = res.numpy()[0], ref.numpy()[0]
    finally:
        for b in (g, ref, res, buf, red):
            b.free()
    expect = parts.max() if op == "max" else parts.sum()
    assert got == want == expect


def test_graph_holds_buffers_and_replays_tile_range(dr):
    """A captured graph keeps raw pointers to the segment's tile-prefix
    buffer: while it is alive a call that would grow that buffer is refused
    (not freed under the graph), and allowed again once it is destroyed.  The
    tile range a captured drhip_reduce_tiles describes takes effect when the
    graph is launched: before the launch an eager tile scan of the range
    reduced before the capture still works, after it only the captured
    range is accepted -- and scans correctly from the replayed prefixes."""
    dr.finalize()
    dr.init([0])  # fresh segment: workspace and tile buffer not yet grown
    na, nb, nbig = 70000, 50000, (1 << 24) + 5
    xa = make_input(np.int32, "plus", na, seed=5)
    xb = make_input(np.int32, "plus", nb, seed=6)
    a, b = dr.DeviceArray(0, na, np.int32, host=xa), dr.DeviceArray(0, nb, np.int32, host=xb)
    da, db = dr.DeviceArray(0, na, np.int32), dr.DeviceArray(0, nb, np.int32)
    big = dr.DeviceArray(0, nbig, np.int32)
    red = dr.DeviceArray(0, 1, np.int32)
    ge = None
    try:
        dr.reduce_tiles_async(0, np.int32, "plus", a.ptr, na, red.ptr)
        dr.sync(0)
        dr.graph_begin(0)
        try:
            dr.reduce_tiles_async(0, np.int32, "plus", b.ptr, nb, red.ptr)
            dr.scan_tiles_async(0, np.int32, "plus", b.ptr, db.ptr, nb)
        finally:
            ge = dr.graph_end(0)
        # nothing replayed yet: the buffer still holds a's prefixes
        with pytest.raises(dr.DrhipError):
            dr.scan_tiles_async(0, np.int32, "plus", b.ptr, db.ptr, nb)
        dr.scan_tiles_async(0, np.int32, "plus", a.ptr, da.ptr, na)
        assert np.array_equal(da.numpy(), np.cumsum(xa.astype(np.int64)).astype(np.int32))
        # growing the tile buffer under the live graph is refused
        with pytest.raises(dr.DrhipError, match="graph"):
            dr.reduce_tiles_async(0, np.int32, "plus", big.ptr, nbig, red.ptr)
        dr.graph_launch(0, ge)
        dr.sync(0)
        assert np.array_equal(db.numpy(), np.cumsum(xb.astype(np.int64)).astype(np.int32))
        with pytest.raises(dr.DrhipError):
            dr.scan_tiles_async(0, np.int32, "plus", a.ptr, da.ptr, na)
        dr.scan_tiles_async(0, np.int32, "plus", b.ptr, da.ptr, nb)
        assert np.array_equal(da.numpy()[:nb], np.cumsum(xb.astype(np.int64)).astype(np.int32))
        dr.graph_destroy(ge)
        ge = None
        dr.reduce_tiles_async(0, np.int32, "plus", big.ptr, nbig, red.ptr)  # grows now
        dr.sync(0)
    finally:
        if ge is not None:
            dr.graph_destroy(ge)
        for buf in (a, b, da, db, big, red):
            buf.free()
        dr.finalize()
        dr.init([0])


def test_scan_tiles_debug_check_catches_changed_input(dr, monkeypatch):
    """DRHIP_CHECK_TILES=1 (debug mode): the tile scan of a range written
    since its drhip_reduce_tiles -- same pointer, size, dtype and op, so the
    range check passes -- is reported by drhip_sync instead of silently
    scanning with stale prefixes; an unchanged range scans as usual."""
    monkeypatch.setenv("DRHIP_CHECK_TILES", "1")
    dr.finalize()
    dr.init([0])
    n = (1 << 20) + 3
    x = make_input(np.int32, "plus", n, seed=8)
    src, dst, red = dr.DeviceArray(0, n, np.int32, host=x), dr.DeviceArray(0, n, np.int32), dr.DeviceArray(0, 1, np.int32)
    try:
        dr.reduce_tiles_async(0, np.int32, "plus", src.ptr, n, red.ptr)
        dr.scan_tiles_async(0, np.int32, "plus", src.ptr, dst.ptr, n)
        assert np.array_equal(dst.numpy(), np.cumsum(x.astype(np.int64)).astype(np.int32))
        dr.reduce_tiles_async(0, np.int32, "plus", src.ptr, n, red.ptr)
        y = x.copy()
        y[n // 2] += 1
        dr.h2d(0, src.ptr, y)
        dr.scan_tiles_async(0, np.int32, "plus", src.ptr, dst.ptr, n)
        with pytest.raises(dr.DrhipError, match="changed since"):
            dr.sync(0)
    finally:
        for b in (src, dst, red):
            b.free()
        monkeypatch.delenv("DRHIP_CHECK_TILES")
        dr.finalize()
        dr.init([0])


def shp_scan_via_abi(dr, oracle, x, n_out, nseg, op, init):
    """The shp layer's multi-segment algorithm (see dr/shp/algorithms/
    inclusive_scan.hpp in this repo) driven through the C-ABI from Python:
    zipped pieces, per-piece totals (reduce), host exclusive prefix of the
    totals, then one carry-in scan per piece."""
    dt = x.dtype
    lens_in = oracle.dv_segments(x.size, nseg)
    lens_out = oracle.dv_segments(n_out, nseg)
    pieces, r_in, r_out = oracle.zip_pieces(lens_in, lens_out)
    segs_out = [dr.DeviceArray(s, max(ln, 1), dt) for s, ln in enumerate(lens_out)]
    segs_in = []
    base = 0
    for s, ln in enumerate(lens_in):
        segs_in.append(dr.DeviceArray(s, max(ln, 1), dt, host=x[base:base + ln]))
        base += ln
    # piece addresses
    addr = []
    off_in = [0] * nseg
    off_out = [0] * nseg
    for ln, ri, ro in zip(pieces, r_in, r_out):
        addr.append((ri, segs_in[ri].at(off_in[ri]), segs_out[ro].at(off_out[ro]), ln))
        off_in[ri] += ln
        off_out[ro] += ln
    # phase 1: totals of every piece but the last
    acc = dr.ACC_OF[dr.DTYPES[dt]]
    totals = []
    for k, (seg, pi, po, ln) in enumerate(addr[:-1]):
        t = dr.DeviceArray(seg, 1, acc)
        dr.reduce_async(seg, dt, op, pi, ln, t.ptr)
        totals.append(t)
    carry = []
    run = None
    for k, t in enumerate(totals):
        v = t.numpy()[0]
        if k == 0 and init is not None:
            v = _op(op, acc(init), v)
        run = v if run is None else _op(op, run, v)
        carry.append(run)
        t.free()
    for k, (seg, pi, po, ln) in enumerate(addr):
        dr.scan_async(seg, dt, op, pi, po, ln, init=init if k == 0 else None,
                      carry=None if k == 0 else carry[k - 1])
    dr.sync()
    out = np.concatenate([s.numpy()[:ln] for s, ln in zip(segs_out, lens_out)])[:x.size]
    for b in segs_in + segs_out:
        b.free()
    return out


@pytest.mark.parametrize("nseg", [1, 3])
def test_inclusive_scan_known_answers(dr, oracle, nseg):
    """ShpTests.InclusiveScan's six lrand48 blocks (algorithms.cpp:61-149) on
    1 and 3 duplicated segments (the shp / shp-3 registrations)."""
    g = json.load(open(GOLDEN))["inclusive_scan"]
    dr.finalize()
    dr.init([0] * nseg)
    try:
        for blk in g["blocks"]:
            x = np.array(blk["input"], dtype=np.int32)
            n_out = g["n"] if blk["layout"] == "inplace" else g["out_size"]
            got = shp_scan_via_abi(dr, oracle, x, n_out, nseg, blk["op"], blk["init"])
            assert got.tolist() == blk["expected"]
    finally:
        dr.finalize()
        dr.init([0])


def test_scan_f32_2pow28_tolerance(dr, oracle):
    """fp32 U[0,1) at 2^28: per-element rel err <= 1e-5 vs the fp64 prefix
    (needs the fp64 inter-tile carries)."""
    n = 1 << 28
    x = np.random.default_rng(1).random(n, dtype=np.float32)
    src = dr.DeviceArray(0, n, np.float32, host=x)
    dst = dr.DeviceArray(0, n, np.float32)
    dr.scan_async(0, np.float32, "plus", src.ptr, dst.ptr, n)
    got = dst.numpy()
    ref = oracle.scan_exact_f32(x)
    err = np.max(np.abs(got - ref) / np.maximum(ref, 1e-30))
    assert err <= FP_RTOL, err
    src.free()
    dst.free()
