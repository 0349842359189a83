"""GPU: the segment allocator's contract (include/drhip.h drhip_malloc /
drhip_free; the reference's device_allocator, shp/allocators.hpp:45-72).

Round 5 made hipMalloc the default (the stream-ordered pool is opt-in,
profiles/r05_pool_stress.txt) and made drhip_free refuse a pointer that is
not a live drhip_malloc block, so a double free cannot release a block
another container has been handed since."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_malloc_roundtrip_and_double_free_refused(dr):
    n = (1 << 20) + 3
    x = np.arange(n, dtype=np.uint32) * np.uint32(2654435761)
    p = dr.malloc(0, x.nbytes)
    dr.h2d(0, p, x)
    assert np.array_equal(dr.d2h(0, p, n, np.uint32), x)
    dr.free(0, p)
    dr.sync(0)
    with pytest.raises(dr.DrhipError):
        dr.free(0, p)  # no longer a live block


def test_free_of_foreign_pointer_refused(dr):
    p = dr.malloc(0, 4096)
    try:
        with pytest.raises(dr.DrhipError):
            dr.free(0, p + 256)  # inside a live block, but not one
    finally:
        dr.free(0, p)


def test_reused_blocks_keep_their_contents(dr):
    """Allocate / write / free in a loop with sizes that straddle 4 MiB
    boundaries, every block read back intact (the pattern under which the
    pool's copies went wrong, in miniature)."""
    rng = np.random.default_rng(5)
    live = []
    for i in range(24):
        n = int(rng.integers(1 << 18, 3 << 20))
        x = rng.integers(0, 1 << 32, size=n, dtype=np.uint64).astype(np.uint32)
        p = dr.malloc(0, x.nbytes)
        dr.h2d(0, p, x)
        live.append((p, x))
        if len(live) > 3:
            q, y = live.pop(0)
            assert np.array_equal(dr.d2h(0, q, y.size, np.uint32), y), f"block {i} changed"
            dr.free(0, q)
    for q, y in live:
        assert np.array_equal(dr.d2h(0, q, y.size, np.uint32), y)
        dr.free(0, q)
    dr.sync(0)
