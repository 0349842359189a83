"""N > 1 host logic of the per-GPU-process path (dr_dist.py) on CPU: the
same combine / splitting / exchange code bench.py runs over RCCL, driven by
world_size 2 and 3 `gloo` process groups with numpy stand-ins for the local
kernels (the reference tests multi-rank without a cluster the same way:
several processes on one host, test/gtest/mhp/CMakeLists.txt:27-33).
Results are compared with the oracle's single-range algorithms."""
import os
import socket
import sys
import traceback

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "distributed-ranges_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, case, q):
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import dr_dist
        out = CASES[case](rank, world, dr_dist)
        q.put((rank, "ok", out))
    except Exception:
        q.put((rank, "err", traceback.format_exc()))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def run(case, world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, case, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = {}
    for _ in range(world):
        r, st, out = q.get(timeout=120)
        assert st == "ok", out
        res[r] = out
    for p in ps:
        p.join(timeout=60)
    return [res[r] for r in range(world)]


# ---------------------------------------------------------------- cases

def _segment(n, world, rank):
    s = (n + world - 1) // world
    return rank * s, min(n, (rank + 1) * s)


def case_reduce(rank, world, D):
    n = 1001
    x = np.arange(n, dtype=np.int64) * 7 - 300
    lo, hi = _segment(n, world, rank)
    part = torch.tensor([x[lo:hi].sum()], dtype=torch.int64)
    return int(D.reduce_partials(part, "plus", init=5).item())


def case_scan(rank, world, D):
    import oracle as O
    n = 100
    rng = np.random.default_rng(0)
    x = rng.integers(0, 100, n).astype(np.int32)
    lo, hi = _segment(n, world, rank)
    seg = x[lo:hi]
    total = torch.tensor([int(seg.astype(np.int64).sum())], dtype=torch.int64)
    carry, has = D.scan_carry(total, "plus")
    local = np.cumsum(seg.astype(np.int64))
    if has:
        local = local + int(carry.item())
    return local.astype(np.int32), O.shp_scan(x, [n], "plus")


def case_sort(rank, world, D):
    rng = np.random.default_rng(rank + 10)
    n_local = 5000 + 37 * rank
    keys = torch.from_numpy(rng.integers(-50, 50, n_local).astype(np.int32))  # heavy ties
    _, to_bits, _ = D.key_bits(np.int32)

    def local_sort(t):
        t.copy_(torch.from_numpy(np.sort(t.numpy())))

    def count_below(t, spl):
        b = to_bits(t.numpy())
        return np.searchsorted(b, to_bits(np.asarray(spl, np.int32)), side="left").astype(np.int64)

    allk = [torch.zeros(5000 + 37 * r, dtype=torch.int32) for r in range(world)]
    for r in range(world):
        allk[r].copy_(torch.from_numpy(np.random.default_rng(r + 10).integers(-50, 50, 5000 + 37 * r).astype(np.int32)))
    out = D.dist_sort(keys, local_sort, count_below)
    return out.numpy(), np.concatenate([a.numpy() for a in allk])


def case_sort_merge(rank, world, D):
    """dist_sort with the merge destination step: the offsets it passes must
    delimit `world` sorted runs (one per source rank) covering the segment."""
    rng = np.random.default_rng(rank + 10)
    keys = torch.from_numpy(rng.integers(-50, 50, 5000 + 37 * rank).astype(np.int32))
    _, to_bits, _ = D.key_bits(np.int32)
    seen = []

    def local_sort(t):
        t.copy_(torch.from_numpy(np.sort(t.numpy())))

    def merge_runs(t, offs):
        x = t.numpy()
        assert len(offs) == world + 1 and offs[0] == 0 and offs[-1] == x.size
        for a, b in zip(offs[:-1], offs[1:]):
            assert np.all(np.diff(x[a:b]) >= 0)
        seen.append(True)
        t.copy_(torch.from_numpy(np.sort(x)))

    def count_below(t, spl):
        b = to_bits(t.numpy())
        return np.searchsorted(b, to_bits(np.asarray(spl, np.int32)), side="left").astype(np.int64)

    allk = [np.random.default_rng(r + 10).integers(-50, 50, 5000 + 37 * r).astype(np.int32) for r in range(world)]
    out = D.dist_sort(keys, local_sort, count_below, merge_runs=merge_runs)
    assert seen == [True]
    return out.numpy(), np.concatenate(allk)


def case_sort_float(rank, world, D):
    rng = np.random.default_rng(rank)
    keys = torch.from_numpy((rng.standard_normal(3000) * 100).astype(np.float32))
    _, to_bits, _ = D.key_bits(np.float32)

    def local_sort(t):
        t.copy_(torch.from_numpy(np.sort(t.numpy())))

    def count_below(t, spl):
        return np.searchsorted(to_bits(t.numpy()), to_bits(np.asarray(spl, np.float32)), side="left").astype(np.int64)

    mine = keys.numpy().copy()
    out = D.dist_sort(keys, local_sort, count_below)
    return out.numpy(), mine


def case_gather_x(rank, world, D):
    x = torch.arange(4, dtype=torch.float32) + 10 * rank
    return D.gather_x(x).numpy()


def case_halo(rank, world, D):
    import oracle as O
    n, r = 30, 1
    a = np.arange(n, dtype=np.int32) * 3 + 1
    lo, hi = _segment(n, world, rank)
    buf = torch.zeros(hi - lo + 2 * r, dtype=torch.int32)
    buf[r:r + hi - lo] = torch.from_numpy(a[lo:hi])
    D.halo_exchange(buf, r)
    b = buf.numpy().astype(np.int64)
    out = a[lo:hi].astype(np.int64).copy()
    for i in range(hi - lo):
        g = lo + i
        if r <= g < n - r:
            out[i] = b[i:i + 2 * r + 1].sum()
    ref = a.copy()
    O.lib().orc_stencil1d_i32(O._p(a), O._p(ref), n, r)
    return out.astype(np.int32), ref[lo:hi]


def case_halo_periodic(rank, world, D):
    """Periodic ring, radius 2: halos hold the neighbours' cells modulo the
    ring (rank 0's prev halo = rank w-1's last cells)."""
    n, r = 31, 2
    a = np.arange(n, dtype=np.int32) * 5 - 7
    lo, hi = _segment(n, world, rank)
    buf = torch.zeros(hi - lo + 2 * r, dtype=torch.int32)
    buf[r:r + hi - lo] = torch.from_numpy(a[lo:hi])
    D.halo_exchange(buf, r, periodic=True)
    want = np.concatenate([a[np.arange(lo - r, lo) % n], a[lo:hi], a[np.arange(hi, hi + r) % n]])
    return buf.numpy(), want


CASES = {"reduce": case_reduce, "halo_periodic": case_halo_periodic, "scan": case_scan, "sort": case_sort, "sort_merge": case_sort_merge,
         "sort_float": case_sort_float,
         "gather_x": case_gather_x, "halo": case_halo}


@pytest.mark.parametrize("world", [2, 3])
def test_reduce_partials(world):
    n = 1001
    ref = 5 + int((np.arange(n, dtype=np.int64) * 7 - 300).sum())
    assert run("reduce", world) == [ref] * world


@pytest.mark.parametrize("world", [2, 3])
def test_scan_carry(world):
    res = run("scan", world)
    got = np.concatenate([r[0] for r in res])
    assert np.array_equal(got, res[0][1])


@pytest.mark.parametrize("world", [2, 3])
def test_dist_sort_exact_split(world):
    res = run("sort", world)
    got = np.concatenate([r[0] for r in res])
    assert np.array_equal(got, np.sort(res[0][1]))
    for rank, r in enumerate(res):  # every rank keeps its key count
        assert r[0].size == 5000 + 37 * rank


@pytest.mark.parametrize("world", [2, 3])
def test_dist_sort_merge_runs(world):
    res = run("sort_merge", world)
    got = np.concatenate([r[0] for r in res])
    assert np.array_equal(got, np.sort(res[0][1]))


def test_dist_sort_float():
    res = run("sort_float", 2)
    got = np.concatenate([r[0] for r in res])
    assert np.array_equal(got, np.sort(np.concatenate([r[1] for r in res])))


def test_gather_x():
    res = run("gather_x", 2)
    for r in res:
        assert np.array_equal(r, np.array([0, 1, 2, 3, 10, 11, 12, 13], np.float32))


@pytest.mark.parametrize("world", [2, 3])
def test_halo_exchange_stencil(world):
    res = run("halo", world)
    for got, ref in res:
        assert np.array_equal(got, ref)


@pytest.mark.parametrize("world", [2, 3])
def test_halo_exchange_periodic(world):
    """The message order drhip_halo_exchange uses (sends reverse then
    forward, receives next halo then prev halo), on a periodic ring; at
    world 2 both neighbours are the same peer."""
    for got, want in run("halo_periodic", world):
        assert np.array_equal(got, want)
