"""CPU tests: pin the oracle (oracle/liboracle.so) to the reference's own
known answers (tests/golden/shp_known_answers.json, generated independently
by tests/golden/make_golden.py) and check its host-side semantics."""
import json
import os

import numpy as np
import pytest

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "shp_known_answers.json")


@pytest.fixture(scope="module")
def golden():
    with open(GOLDEN) as f:
        return json.load(f)


# ------------------------------------------------------------ partitioning


@pytest.mark.parametrize("n,p,expect", [
    (10, 1, [10]), (10, 3, [4, 4, 2]), (100, 3, [34, 34, 32]), (200, 3, [67, 67, 66]),
    (9, 3, [3, 3, 3]), (2, 3, [1, 1]), (0, 4, [0]), (1, 8, [1]), (17, 4, [5, 5, 5, 2]),
])
def test_dv_segments(oracle, n, p, expect):
    """distributed_vector.hpp:142 ceil(n/P) + take_segments trimming."""
    assert oracle.dv_segments(n, p) == expect


def test_zip_pieces_misaligned(oracle):
    """InclusiveScan's misaligned case: v(100) zipped with o(200) on 3 devices."""
    pieces, rr, ro = oracle.zip_pieces(oracle.dv_segments(100, 3), oracle.dv_segments(200, 3))
    assert pieces == [34, 33, 1, 32]
    assert rr == [0, 1, 1, 2] and ro == [0, 0, 1, 1]
    assert sum(pieces) == 100


def test_subrange_segments(oracle):
    pieces, ranks = oracle.subrange_segments([4, 4, 2], 3, 9)
    assert pieces == [1, 4, 1] and ranks == [0, 1, 2]


# ------------------------------------------------------- reference answers


@pytest.mark.parametrize("p", [1, 2, 3, 4, 7, 10, 12])
def test_reduce_basic_known_answer(oracle, golden, p):
    """ShpTests.ReduceBasic (algorithms.cpp:39-59): iota(10) over n=10 -> 145,
    for every segment count including length-1 segments (reduce.hpp:69-71)."""
    g = golden["reduce_basic"]
    x = np.arange(g["start"], g["start"] + g["n"], dtype=np.int32)
    assert oracle.shp_reduce(x, oracle.dv_segments(g["n"], p), g["init"]) == g["expected"]


@pytest.mark.parametrize("p", [1, 3])
def test_inclusive_scan_known_answers(oracle, golden, p):
    """ShpTests.InclusiveScan (algorithms.cpp:61-149): the six lrand48 blocks,
    aligned (in place) and misaligned (o of size 2n) on 1 and 3 devices
    (the shp and shp-3 registrations, test/gtest/shp/CMakeLists.txt:28-30)."""
    g = golden["inclusive_scan"]
    draws = oracle.lrand48_mod(g["n"] * 6, 100, reseed=True)
    for bi, blk in enumerate(g["blocks"]):
        x = np.array(blk["input"], dtype=np.int32)
        assert np.array_equal(x, draws[bi * 100:(bi + 1) * 100]), "lrand48 stream"
        lens_in = oracle.dv_segments(g["n"], p)
        lens_out = lens_in if blk["layout"] == "inplace" else oracle.dv_segments(g["out_size"], p)
        pieces, _, _ = oracle.zip_pieces(lens_in, lens_out)
        got = oracle.shp_scan(x, pieces, blk["op"], blk["init"])
        assert got.tolist() == blk["expected"], (bi, blk["op"])


def test_inclusive_scan_product_wraps(oracle, golden):
    """Block 2 (multiplies, init 12) has no zero and overflows int32: the
    oracle must wrap exactly like the reference's int arithmetic."""
    blk = golden["inclusive_scan"]["blocks"][2]
    assert 0 not in blk["input"][:50]
    big = 12
    for v in blk["input"][:12]:
        big *= v
    assert big > 2**31  # genuinely overflows


def test_mhp_reduce_known_answer(oracle, golden):
    g = golden["mhp_reduce"]
    x = np.arange(g["start"], g["start"] + g["n"], dtype=np.int32)
    for ranks in (1, 2, 3, 4):
        assert oracle.mhp_reduce_i32(x, ranks, g["init"]) == g["expected"]


def test_mhp_stencil_known_answer(oracle, golden):
    g = golden["mhp_stencil"]
    x = np.arange(g["in_start"], g["in_start"] + g["n"], dtype=np.int32)
    out = np.full(g["n"], g["out_fill"], dtype=np.int32)
    assert oracle.stencil_mhp_test_op(x, g["radius"], out).tolist() == g["expected"]


@pytest.mark.parametrize("ranks", [1, 2, 3, 4])
def test_stencil_1d_known_answer(oracle, golden, ranks):
    """examples/mhp/stencil-1d.cpp with halo exchange on 1-4 ranks."""
    g = golden["stencil_1d"]
    a = np.arange(g["a_start"], g["a_start"] + g["n"], dtype=np.int32)
    b = np.full(g["n"], g["b_fill"], dtype=np.int32)
    A, B, cur = oracle.stencil1d_mhp_steps(a, b, ranks, g["steps"])
    res = (A, B)[cur]
    assert res[1:-1].tolist() == g["expected_interior"]


# ---------------------------------------------------- oracle self-checks


def test_scan_matches_numpy_wrapping(oracle):
    rng = np.random.default_rng(1)
    x = rng.integers(-2**31, 2**31, size=5000, dtype=np.int64).astype(np.int32)
    pieces = [1000, 1, 2999, 1000]
    got = oracle.shp_scan(x, pieces, "plus")
    ref = np.cumsum(x.astype(np.uint32), dtype=np.uint32).astype(np.int32)
    assert np.array_equal(got, ref)


def test_reduce_exact_f32(oracle):
    rng = np.random.default_rng(2)
    x = rng.random(1 << 16, dtype=np.float32)
    assert abs(oracle.reduce_exact(x) - float(np.sum(x.astype(np.float64)))) < 1e-9 * (1 << 16)


def test_csr_generators(oracle):
    rp, ci, v = oracle.csr_gen("banded", 0, 50, 50, 1)
    assert rp[0] == 0 and rp[-1] == ci.size
    for i in range(50):
        cols = ci[rp[i]:rp[i + 1]]
        assert cols.tolist() == list(range(max(0, i - 4), min(50, i + 6)))
    rp2, ci2, v2 = oracle.csr_gen("banded", 20, 10, 50, 1)
    assert np.array_equal(ci2, ci[rp[20]:rp[30]]) and np.array_equal(v2, v[rp[20]:rp[30]])
    rp, ci, v = oracle.csr_gen("random", 0, 64, 1000, 7, k=10)
    for i in range(64):
        cols = ci[rp[i]:rp[i + 1]]
        assert len(cols) == 10 and np.all(np.diff(cols) > 0) and cols.max() < 1000
    assert np.all((v >= 0) & (v < 1))


def test_spmv_matches_dense(oracle):
    rp, ci, v = oracle.csr_gen("random", 0, 40, 30, 3, k=5)
    x = np.random.default_rng(3).random(30, dtype=np.float32)
    dense = np.zeros((40, 30))
    for i in range(40):
        dense[i, ci[rp[i]:rp[i + 1]]] = v[rp[i]:rp[i + 1]]
    y0 = np.ones(40, dtype=np.float32)
    assert np.allclose(oracle.csr_spmv(rp, ci, v, x, y0), dense @ x + 1.0, rtol=1e-12)


def test_sort(oracle):
    x = np.random.default_rng(4).integers(0, 2**32, size=10000, dtype=np.uint64).astype(np.uint32)
    assert np.array_equal(oracle.sort(x), np.sort(x))


def test_mhp_scan_threads(oracle):
    x = np.random.default_rng(5).random(100003, dtype=np.float32)
    ref = np.cumsum(x.astype(np.float64))
    for ranks, th in ((1, 1), (4, 2), (7, 4)):
        got = oracle.mhp_scan(x, ranks, th)
        assert np.max(np.abs(got - ref) / ref) < 1e-6
    xi = np.random.default_rng(6).integers(-1000, 1000, size=50001).astype(np.int32)
    assert np.array_equal(oracle.mhp_scan(xi, 5, 3), np.cumsum(xi.astype(np.int64)).astype(np.int32))


def test_csr_density_generator_properties(oracle):
    """Density generator: floor(density*m*n) entries (generate_random.hpp:37), rows sorted and distinct."""
    m, n, d = 500, 300, 0.03
    rp, ci, va = oracle.csr_gen_density(0, m, m, n, d, 9)
    assert rp[-1] == int(d * m * n) == ci.size
    assert np.all(np.diff(rp) >= 0) and np.max(np.diff(rp)) - np.min(np.diff(rp)) <= 1
    for r in range(m):
        row = ci[rp[r]:rp[r + 1]]
        assert np.all(np.diff(row) > 0) and (row.size == 0 or (row[0] >= 0 and row[-1] < n))
    assert np.all((va >= 0) & (va < 1))
    # tiles concatenate to the whole matrix
    a = oracle.csr_gen_density(0, 200, m, n, d, 9)
    b = oracle.csr_gen_density(200, 300, m, n, d, 9)
    assert np.array_equal(np.concatenate([a[1], b[1]]), ci)
    assert np.array_equal(np.concatenate([a[0][:-1], b[0] + a[0][-1]]), rp)
    _, _, iv = oracle.csr_gen_density(0, m, m, n, d, 9, int_values=True)
    assert set(np.unique(iv)) <= {0.0, 1.0}


@pytest.mark.parametrize("n", [0, 1, 7, 1000, 65537])
def test_radix_sort_u32_equals_qsort(oracle, n):
    """The O(n) uint32 sort used for the full-size C3 checks gives the same
    bytes as the std::less qsort restatement."""
    x = np.random.default_rng(n).integers(0, 1 << 32, n, dtype=np.uint32)
    x[: n // 3] = x[n // 2] if n else 0  # ties
    assert np.array_equal(oracle.sort_u32_large(x), oracle.sort(x))


@pytest.mark.parametrize("threads", [1, 3, 8])
@pytest.mark.parametrize("n", [0, 5, 1000, (1 << 20) + 17])
def test_radix_sort_u32_par_equals_serial(oracle, n, threads):
    """orc_radix_sort_u32_par (the 2^31-key C3 checker) == the serial radix."""
    x = oracle.hash_u32(n, seed=7, start=3)
    x[: n // 4] = x[n // 2] if n else 0
    assert np.array_equal(oracle.sort_u32_large_par(x, threads), oracle.sort_u32_large(x))


def test_hash_u32_is_splitmix64_high_word(oracle):
    """The C3 key generator: high word of splitmix64(seed + i), restated in Python."""
    M = (1 << 64) - 1

    def sm(z):
        z = (z + 0x9E3779B97F4A7C15) & M
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M
        return (z ^ (z >> 31)) >> 32
    got = oracle.hash_u32(100, seed=5, start=1 << 33)
    assert got.tolist() == [sm(5 + (1 << 33) + i) for i in range(100)]
