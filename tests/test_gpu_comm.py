"""GPU tests of the RCCL layer behind the C-ABI (csrc/comm.hip) on ONE rank.

The box has one GPU and RCCL refuses two ranks on one device, so the
multi-rank message pattern is covered here by what a single rank can check
-- self-sends that go through the same grouped ncclSend/ncclRecv code (the
periodic halo with one rank wraps onto itself, a one-peer all-to-all), and
the collectives' identities at nranks = 1 -- and by the world-2/3 gloo tests
of the same host logic (tests/test_dist_gloo.py).  Reference semantics:
details/halo.hpp:336-387 (span_halo groups), communicator.hpp:51-56."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def comm(dr):
    uid = dr.comm_unique_id()
    assert len(uid) == dr.COMM_ID_BYTES
    dr.comm_init_rank(0, 1, 0, uid)
    yield dr
    dr.comm_destroy(0)


def test_comm_rank(comm):
    assert comm.comm_rank(0) == (0, 1)


@pytest.mark.parametrize("dtype", [np.int32, np.uint32, np.int64, np.float32, np.float64])
@pytest.mark.parametrize("op", ["plus", "mul", "min", "max"])
def test_allreduce_one_rank(comm, dtype, op):
    x = (np.arange(1, 1001) % 97).astype(dtype)
    src = comm.DeviceArray(0, x.size, dtype, host=x)
    dst = comm.DeviceArray(0, x.size, dtype)
    comm.allreduce(0, dtype, op, src.ptr, dst.ptr, x.size)
    assert np.array_equal(dst.numpy(), x)
    src.free()
    dst.free()


def test_allgather_and_gather_one_rank(comm):
    x = np.random.default_rng(1).integers(0, 255, 4099, dtype=np.uint8)
    src = comm.DeviceArray(0, x.size, np.uint8, host=x)
    dst = comm.DeviceArray(0, x.size, np.uint8)
    comm.allgather(0, src.ptr, dst.ptr, x.size)
    assert np.array_equal(dst.numpy(), x)
    dst2 = comm.DeviceArray(0, x.size, np.uint8)
    comm.gather(0, src.ptr, dst2.ptr, x.size, 0)
    assert np.array_equal(dst2.numpy(), x)
    for b in (src, dst, dst2):
        b.free()


def test_alltoallv_self(comm):
    """One peer (itself): a block at an offset goes to an offset."""
    x = np.arange(1000, dtype=np.int32)
    src = comm.DeviceArray(0, 1000, np.int32, host=x)
    dst = comm.DeviceArray(0, 1000, np.int32, host=np.full(1000, -1, np.int32))
    comm.alltoallv(0, src.ptr, [400 * 4], [100 * 4], dst.ptr, [400 * 4], [500 * 4])
    got = dst.numpy()
    assert np.array_equal(got[500:900], x[100:500])
    assert np.all(got[:500] == -1) and np.all(got[900:] == -1)
    src.free()
    dst.free()


@pytest.mark.parametrize("n_owned,r", [(10, 1), (10, 4), (1 << 20, 3), (7, 7)])
def test_halo_periodic_one_rank(comm, oracle, n_owned, r):
    """Periodic with one rank: rank-1 = rank+1 = itself, so the prev halo
    gets the last r owned cells and the next halo the first r (the wrap of
    halo.hpp's owned/halo groups), through the same grouped send/recv
    order a 2-rank periodic ring uses."""
    x = np.random.default_rng(n_owned).integers(-1000, 1000, n_owned + 2 * r).astype(np.int32)
    buf = comm.DeviceArray(0, x.size, np.int32, host=x)
    comm.halo_exchange(0, buf.ptr, n_owned, 4, r, r, periodic=True)
    got = buf.numpy()
    want = x.copy()
    want[:r] = x[n_owned:n_owned + r]            # last r owned cells
    want[r + n_owned:] = x[r:2 * r]              # first r owned cells
    assert np.array_equal(got, want)
    buf.free()


def test_halo_nonperiodic_one_rank_is_noop_and_rows(comm):
    x = np.arange(30, dtype=np.float32)
    buf = comm.DeviceArray(0, 30, np.float32, host=x)
    comm.halo_exchange(0, buf.ptr, 28, 4, 1, 1, periodic=False)
    assert np.array_equal(buf.numpy(), x)
    buf.free()
    # 2-D row block: a cell is one row of nx floats
    nx, rows = 64, 9
    g = np.random.default_rng(2).random((rows + 2) * nx, dtype=np.float32)
    b2 = comm.DeviceArray(0, g.size, np.float32, host=g)
    comm.halo_exchange(0, b2.ptr, rows, 4 * nx, 1, 1, periodic=True)
    got = b2.numpy().reshape(rows + 2, nx)
    want = g.reshape(rows + 2, nx).copy()
    want[0] = want[rows]
    want[rows + 1] = want[1]
    assert np.array_equal(got, want)
    b2.free()


def test_halo_rejects_asymmetric(comm):
    buf = comm.DeviceArray(0, 16, np.int32)
    with pytest.raises(comm.DrhipError):
        comm.halo_exchange(0, buf.ptr, 10, 4, 2, 1, periodic=True)
    buf.free()


def test_comm_init_all_single_segment(dr):
    """shp model: one communicator per segment of this process."""
    dr.comm_init_all()
    assert dr.comm_rank(0) == (0, 1)
    x = np.arange(64, dtype=np.float64)
    src = dr.DeviceArray(0, 64, np.float64, host=x)
    dst = dr.DeviceArray(0, 64, np.float64)
    dr.allreduce(0, np.float64, "plus", src.ptr, dst.ptr, 64)
    assert np.array_equal(dst.numpy(), x)
    src.free()
    dst.free()
    dr.comm_destroy(0)


# -------------------------- dr_dist.DrhipTransport over the one-rank comm
def test_drhip_transport_one_rank(dr):
    """bench.py's N > 1 transport object on the real RCCL C-ABI, one rank:
    all_gather of one block, a one-peer all_to_all (self send/recv through
    drhip_alltoallv's grouped calls) and the periodic halo wrap, with torch
    tensors on the segment stream."""
    import torch
    import dr_dist
    comm = dr
    torch.zeros(1, device="cuda")  # torch's device state first, as bench.py orders it
    torch.cuda.synchronize()
    comm.comm_init_rank(0, 1, 0, comm.comm_unique_id())
    stream = torch.cuda.ExternalStream(comm.stream(0))
    t = dr_dist.DrhipTransport(0, stream=stream)
    assert t.world() == (1, 0)
    with torch.cuda.stream(stream):
        x = torch.arange(10, dtype=torch.float64, device="cuda")
        out = torch.empty(10, dtype=torch.float64, device="cuda")
        t.all_gather_into(out, x)
        k = torch.arange(1000, dtype=torch.int32, device="cuda") * 3
        ko = torch.empty_like(k)
        t.all_to_all(ko, k, [1000], [1000])
        buf = torch.arange(14, dtype=torch.int32, device="cuda")
        t.halo(buf, 2, True)
    torch.cuda.synchronize()
    assert torch.equal(out.cpu(), x.cpu())
    assert torch.equal(ko.cpu(), k.cpu())
    b = list(range(14))
    assert buf.cpu().tolist() == [b[10], b[11]] + b[2:12] + [b[2], b[3]]
    comm.comm_destroy(0)


@pytest.mark.parametrize("dtype", [np.float64, np.int32, np.int64, np.uint32, np.uint64])
@pytest.mark.parametrize("op", ["plus", "mul", "min", "max"])
@pytest.mark.parametrize("w", [1, 2, 5, 8])
def test_fold_partials(dr, dtype, op, w):
    """drhip_fold_partials: left folds in segment order (reduce.hpp:81-83)
    of w partials, the total and the carry of every rank, bit-exact vs the
    same loop in numpy (wrapping integers, fp64 in order)."""
    rng = np.random.default_rng(w)
    if np.dtype(dtype).kind == "f":
        p = (rng.standard_normal(w) * 10.0 ** rng.integers(-8, 8, w)).astype(dtype)
    else:
        info = np.iinfo(dtype)
        p = rng.integers(info.min, info.max, w, endpoint=True, dtype=dtype)
    f = {"plus": np.add, "mul": np.multiply, "min": np.minimum, "max": np.maximum}[op]
    src = dr.DeviceArray(0, w, dtype, host=p)
    for rank in range(w):
        res = dr.DeviceArray(0, 1, dtype)
        car = dr.DeviceArray(0, 1, dtype, host=np.zeros(1, dtype))
        dr.fold_partials_async(0, dtype, op, src.ptr, w, rank, res.ptr, car.ptr)
        with np.errstate(over="ignore"):
            acc = p[0]
            carry = None
            for k in range(1, w):
                if k == rank:
                    carry = acc
                acc = f(acc, p[k]).astype(dtype)
        got = res.numpy()[0]
        assert got.tobytes() == np.asarray(acc, dtype).tobytes()
        if rank:
            assert car.numpy()[0].tobytes() == np.asarray(carry, dtype).tobytes()
        res.free()
        car.free()
    src.free()
