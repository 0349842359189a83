"""GPU parity: drhip_reduce / drhip_dot (C-ABI) against the oracle.

Integers are bit-exact (wrapping two's complement); floats within a
relative tolerance of the fp64-compensated oracle sum (1e-5 at every size,
BASELINE.json north_star)."""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

DTYPES = [np.int32, np.uint32, np.int64, np.uint64, np.float32, np.float64]
OPS = ["plus", "mul", "min", "max"]
FP_RTOL = 1e-5


def make_input(dtype, op, n, seed):
    rng = np.random.default_rng(seed)
    dt = np.dtype(dtype)
    if dt.kind == "f":
        if op == "mul":
            return (1.0 + (rng.random(n) - 0.5) * 1e-3).astype(dt)
        return rng.random(n).astype(dt)
    info = np.iinfo(dt)
    return rng.integers(info.min, info.max, size=n, endpoint=True, dtype=dt)


def check_value(got, ref, dtype):
    if np.dtype(dtype).kind == "f":
        assert abs(got - ref) <= FP_RTOL * max(abs(ref), 1e-30), (got, ref)
    else:
        assert np.array(got).astype(dtype) == np.array(ref).astype(dtype), (got, ref)


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("op", OPS)
@pytest.mark.parametrize("n,offset", [(0, 0), (1, 0), (7, 1), (1000, 3), (4097, 0), (70001, 1),
                                      ((1 << 20) + 3, 2)])
def test_reduce_parity(dr, oracle, dtype, op, n, offset):
    x = make_input(dtype, op, n + offset, seed=n * 7 + offset)
    buf = dr.DeviceArray(0, n + offset, dtype, host=x)
    got = dr.reduce(0, buf.at(offset), n, dtype, op)
    xs = x[offset:]
    if np.dtype(dtype).kind == "f":
        ref = oracle.reduce_exact(xs, {"plus": 0.0, "mul": 1.0, "min": np.inf, "max": -np.inf}[op], op)
        if n == 0:
            assert got == {"plus": 0.0, "mul": 1.0, "min": np.inf, "max": -np.inf}[op]
        else:
            check_value(got, ref, dtype)
    else:
        ident = {"plus": 0, "mul": 1, "min": np.iinfo(dtype).max, "max": np.iinfo(dtype).min}[op]
        ref = oracle.shp_reduce(xs, [n], ident, op) if n else ident
        check_value(got, ref, dtype)
    buf.free()


@pytest.mark.parametrize("nseg", [1, 3, 4, 10, 12])
def test_reduce_basic_known_answer_segments(dr, oracle, nseg):
    """ShpTests.ReduceBasic (algorithms.cpp:39-59) -> 145 through the C-ABI,
    with the shp segment fold (reduce.hpp:60-84) over nseg duplicated
    segments on one GPU (shp-tests.cpp:34-39 device duplication)."""
    golden = json.load(open(os.path.join(os.path.dirname(__file__), "golden",
                                          "shp_known_answers.json")))["reduce_basic"]
    n = golden["n"]
    dr.finalize()
    dr.init([0] * nseg)
    try:
        lens = oracle.dv_segments(n, nseg)
        x = np.arange(golden["start"], golden["start"] + n, dtype=np.int32)
        init = np.int32(golden["init"])
        partials = []
        base = 0
        for s, ln in enumerate(lens):
            seg = dr.DeviceArray(s, ln, np.int32, host=x[base:base + ln])
            if ln == 1:
                init = np.int32(init + seg.numpy()[0])  # host fold (reduce.hpp:69-71)
            elif ln > 1:
                partials.append(dr.reduce(s, seg.ptr, ln, np.int32))
            base += ln
            seg.free()
        for p in partials:
            init = np.int32(init + p)
        assert int(init) == golden["expected"] == oracle.shp_reduce(x, lens, 0)
    finally:
        dr.finalize()
        dr.init([0])


@pytest.mark.parametrize("n", [1 << 28])
def test_reduce_f32_large_tolerance(dr, oracle, n):
    """2^28 fp32 U[0,1): rel err <= 1e-5 vs fp64 compensated."""
    x = np.random.default_rng(11).random(n, dtype=np.float32)
    buf = dr.DeviceArray(0, n, np.float32, host=x)
    got = dr.reduce(0, buf.ptr, n, np.float32)
    ref = oracle.reduce_exact(x)
    assert abs(got - ref) / ref < 1e-6
    ib = dr.DeviceArray(0, n, np.int32, host=(x * 65536).astype(np.int32))
    gi = dr.reduce(0, ib.ptr, n, np.int32)
    assert int(gi) == int(oracle.shp_reduce((x * 65536).astype(np.int32), [n], 0))
    buf.free()
    ib.free()


@pytest.mark.parametrize("dtype", [np.float32, np.float64, np.int32])
@pytest.mark.parametrize("n,offset", [(0, 0), (5, 1), (4099, 0), (1 << 20, 0), (300001, 2)])
def test_dot_parity(dr, oracle, dtype, n, offset):
    """transform_reduce / dot (examples/shp/dot_product.cpp:11-18)."""
    rng = np.random.default_rng(n + 17)
    if np.dtype(dtype).kind == "f":
        x = rng.random(n + offset).astype(dtype)
        y = rng.random(n + offset).astype(dtype)
    else:
        x = rng.integers(-1000, 1000, n + offset).astype(dtype)
        y = rng.integers(-1000, 1000, n + offset).astype(dtype)
    bx = dr.DeviceArray(0, n + offset, dtype, host=x)
    by = dr.DeviceArray(0, n + offset, dtype, host=y)
    acc = np.float64 if np.dtype(dtype).kind == "f" else dtype
    out = dr.DeviceArray(0, 1, acc)
    dr.dot_async(0, dtype, bx.at(offset), by.at(offset), n, out.ptr)
    got = out.numpy()[0]
    ref = oracle.dot(x[offset:], y[offset:])
    if np.dtype(dtype).kind == "f":
        assert abs(got - ref) <= FP_RTOL * max(abs(ref), 1e-30)
    else:
        assert int(got) == int(ref)
    for b in (bx, by, out):
        b.free()


@pytest.mark.parametrize("dtype", [np.float32, np.float64, np.int32])
@pytest.mark.parametrize("n,xo,yo", [(7, 1, 0), (4099, 0, 1), (300001, 1, 2), ((1 << 22) + 3, 1, 0)])
def test_dot_shifted_operands(dr, oracle, dtype, n, xo, yo):
    """dot(x[xo:], y[yo:]) with the two operands at different 16-byte
    alignments (a zipped pair of shifted sub-ranges): the multi-block
    element-load path for y, same result as the aligned path."""
    rng = np.random.default_rng(n + 31)
    if np.dtype(dtype).kind == "f":
        x = rng.random(n + 3).astype(dtype)
        y = rng.random(n + 3).astype(dtype)
    else:
        x = rng.integers(-1000, 1000, n + 3).astype(dtype)
        y = rng.integers(-1000, 1000, n + 3).astype(dtype)
    bx = dr.DeviceArray(0, n + 3, dtype, host=x)
    by = dr.DeviceArray(0, n + 3, dtype, host=y)
    acc = np.float64 if np.dtype(dtype).kind == "f" else dtype
    out = dr.DeviceArray(0, 1, acc)
    dr.dot_async(0, dtype, bx.at(xo), by.at(yo), n, out.ptr)
    got = out.numpy()[0]
    ref = oracle.dot(x[xo:xo + n], y[yo:yo + n])
    if np.dtype(dtype).kind == "f":
        assert abs(got - ref) <= FP_RTOL * max(abs(ref), 1e-30)
    else:
        assert int(got) == int(ref)
    for b in (bx, by, out):
        b.free()


def test_c1_mhp_dot_two_segments(dr, oracle):
    """BASELINE configs[0] shape: dot product of two 2^24-element fp32
    vectors split into 2 segments (the reference runs it on 2 MPI ranks):
    per-segment drhip_dot partials folded in segment order, as
    mhp::reduce gathers them to the root (cpu_algorithms.hpp:102-140), within
    rtol 1e-5 of the fp64 oracle."""
    n = 1 << 24
    rng = np.random.default_rng(1)
    x = rng.random(n, dtype=np.float32)
    y = rng.random(n, dtype=np.float32)
    bx = dr.DeviceArray(0, n, np.float32, host=x)
    by = dr.DeviceArray(0, n, np.float32, host=y)
    out = dr.DeviceArray(0, 2, np.float64)
    half = n // 2
    for k in range(2):
        dr.dot_async(0, np.float32, bx.at(k * half), by.at(k * half), half, out.at(k))
    p = out.numpy()
    got = 0.0 + p[0] + p[1]
    ref = oracle.dot(x, y)
    assert abs(got - ref) <= FP_RTOL * abs(ref)
    for b in (bx, by, out):
        b.free()
