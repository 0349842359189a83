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


class EmulatedDrhipComm:
    """The four calls dr_dist.DrhipTransport makes into libdrhip's RCCL C-ABI
    (drhip_comm_rank / drhip_allgather / drhip_alltoallv /
    drhip_halo_exchange, csrc/comm.hip), emulated over gloo on host memory
    with the same pointer/byte-count arguments and the same message order --
    so the CPU tests run DrhipTransport's own offset and count arithmetic."""

    @staticmethod
    def _view(ptr, nbytes):
        import ctypes
        if nbytes == 0:
            return torch.empty(0, dtype=torch.uint8)
        return torch.frombuffer((ctypes.c_uint8 * int(nbytes)).from_address(int(ptr)), dtype=torch.uint8)

    def comm_rank(self, seg):
        return dist.get_rank(), dist.get_world_size()

    def allgather(self, seg, send, recv, nbytes):
        w = dist.get_world_size()
        dist.all_gather_into_tensor(self._view(recv, w * nbytes), self._view(send, nbytes).clone())

    def alltoallv(self, seg, send, sb, so, recv, rb, ro):
        me, w = dist.get_rank(), dist.get_world_size()
        ops = []
        for r in range(w):  # grouped send/recv per peer, zero-byte pairs skipped
            if r == me:
                if sb[r]:
                    self._view(recv + int(ro[r]), rb[r]).copy_(self._view(send + int(so[r]), sb[r]).clone())
                continue
            if sb[r]:
                ops.append(dist.P2POp(dist.isend, self._view(send + int(so[r]), sb[r]).clone(), r))
            if rb[r]:
                ops.append(dist.P2POp(dist.irecv, self._view(recv + int(ro[r]), rb[r]), r))
        for q in (dist.batch_isend_irecv(ops) if ops else []):
            q.wait()

    def halo_exchange(self, seg, buf, n_owned, cell_bytes, prev, nxt, periodic):
        assert prev == nxt
        me, w = dist.get_rank(), dist.get_world_size()
        hb = prev * cell_bytes
        do_prev, do_next = periodic or me > 0, periodic or me < w - 1
        rprev, rnext = (me - 1) % w, (me + 1) % w
        ops = []  # comm.hip's order: sends [reverse, forward], receives [next halo, prev halo]
        if do_prev:
            ops.append(dist.P2POp(dist.isend, self._view(buf + hb, hb).clone(), rprev))
        if do_next:
            ops.append(dist.P2POp(dist.isend, self._view(buf + n_owned * cell_bytes, hb).clone(), rnext))
            ops.append(dist.P2POp(dist.irecv, self._view(buf + hb + n_owned * cell_bytes, hb), rnext))
        if do_prev:
            ops.append(dist.P2POp(dist.irecv, self._view(buf, hb), rprev))
        for q in dist.batch_isend_irecv(ops):
            q.wait()


def case_bench_graph_phase(rank, world, D, inject_rank):
    """bench.py's graph mode (graph_phase) with rank `inject_rank`'s capture
    failing: every rank must come back with the error instead of one rank
    replaying a graph whose captured collective (here a gloo all_reduce) the
    other never joins -- that would hang, and run()'s queue would time out."""
    sys.path.insert(0, ROOT)
    import bench
    bench.CPU_GROUP = dist.group.WORLD
    if inject_rank is None:
        os.environ.pop("DRHIP_BENCH_FAIL_CAPTURE_RANK", None)
    else:
        os.environ["DRHIP_BENCH_FAIL_CAPTURE_RANK"] = str(inject_rank)

    class FakeTorch:
        tensor = staticmethod(torch.tensor)
        int32 = torch.int32

        class cuda:
            @staticmethod
            def synchronize():
                pass

    launches, destroyed = [], []

    def capture(inject):
        if inject:
            raise RuntimeError("injected capture failure (DRHIP_BENCH_FAIL_CAPTURE_RANK)")
        return "graph"

    def launch(ge):
        dist.all_reduce(torch.ones(1))  # the captured collective
        launches.append(ge)

    def timed(fn):
        for _ in range(3):
            fn()
        return 1.5

    ms, err = bench.graph_phase(FakeTorch, dist, world, rank, capture, launch, destroyed.append, timed)
    return ms, err, len(launches), destroyed


class EmulatedXchgLib:
    """drhip's flag-slot / IPC calls as FlagSlots makes them, on host ints:
    a slot array is an id, its handle the id's bytes, opening a handle gives
    the id back (as a peer mapping would), and the exchange itself is an
    all_gather over gloo of the 8-byte host value at `value`."""

    def __init__(self, rank):
        self.rank, self.freed, self.closed = rank, [], []

    def xchg_alloc(self, seg, w):
        return 1000 + self.rank

    def xchg_free(self, seg, p):
        self.freed.append(p)

    def ipc_handle(self, p):
        return int(p).to_bytes(8, "little") + bytes(56)

    def ipc_open(self, seg, h):
        return int.from_bytes(h[:8], "little")

    def ipc_close(self, seg, p):
        self.closed.append(p)

    def xchg_allgather(self, seg, local, peers, rank, value, gathered, value_bytes=8):
        import ctypes
        assert peers[rank] == local and peers == [1000 + j for j in range(len(peers))]
        src = torch.frombuffer((ctypes.c_uint8 * value_bytes).from_address(value), dtype=torch.uint8).clone()
        out = torch.frombuffer((ctypes.c_uint8 * (value_bytes * len(peers))).from_address(gathered), dtype=torch.uint8)
        dist.all_gather_into_tensor(out, src)


def case_flag_slots(rank, world, D):
    lib = EmulatedXchgLib(rank)
    fs = D.FlagSlots.bootstrap(0, lib=lib)
    out = []
    for dt, v in ((torch.float64, 0.5 + rank), (torch.int32, -7 * rank)):
        g = torch.zeros(world, dtype=dt)
        fs.all_gather_into(g, torch.tensor([v], dtype=dt))
        out.append(g.tolist())
    fs.close()
    return fs.peers, out, lib.closed, lib.freed


def case_flag_slots_open_failure(rank, world, D):
    """FlagSlots.bootstrap when mapping the LAST peer's array fails: the
    error reaches the caller, the peers already mapped are unmapped and the
    local array is freed."""
    class Failing(EmulatedXchgLib):
        def ipc_open(self, seg, h):
            p = super().ipc_open(seg, h)
            if p == 1000 + max(j for j in range(world) if j != rank):
                raise RuntimeError("emulated ipc_open failure")
            return p

    lib = Failing(rank)
    try:
        D.FlagSlots.bootstrap(0, lib=lib)
        raised = False
    except RuntimeError:
        raised = True
    return raised, lib.closed, lib.freed


def case_bench_check_sort(rank, world, D):
    """bench.py's N > 1 sort check on a correct and on two corrupted outputs
    (uint32 keys in int32 tensors, as the bench carries them)."""
    sys.path.insert(0, ROOT)
    import bench
    n = 1000
    g = np.random.default_rng(0).integers(0, 1 << 32, n * world, dtype=np.uint64).astype(np.uint32)
    mine = g[rank * n:(rank + 1) * n]
    srt = np.sort(g)
    good = srt[rank * n:(rank + 1) * n]
    src = torch.from_numpy(mine.view(np.int32).copy())
    res = [bench.check_sort(torch, dist, src, torch.from_numpy(good.view(np.int32).copy()), world)["ok"]]
    # a duplicate in place of a neighbour's key: sorted, bounds ordered, but not the same multiset
    bad = good.copy()
    if rank == 0:
        bad[-1] = bad[-2]
    res.append(bench.check_sort(torch, dist, src, torch.from_numpy(bad.view(np.int32).copy()), world)["ok"])
    # ranks 0 and 1 swap their blocks: every rank locally sorted, multiset
    # intact, but the global ranks of the first / last keys are wrong
    sw = srt[(1 - rank) * n:(2 - rank) * n] if rank < 2 else good
    res.append(bench.check_sort(torch, dist, src, torch.from_numpy(sw.view(np.int32).copy()), world))
    return res


def _worker(rank, world, port, case, q):
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import dr_dist
        if case.endswith("@drhip"):  # the DrhipTransport path, RCCL calls emulated over gloo
            case = case[:-len("@drhip")]
            dr_dist.use(dr_dist.DrhipTransport(0, lib=EmulatedDrhipComm()))
        if case.startswith("bench_graph_phase"):
            arg = case.split(":")[1]
            out = case_bench_graph_phase(rank, world, dr_dist, None if arg == "none" else int(arg))
        else:
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


INIT_ORDER_VALS = [1e16, 1.0, 1.0, 3.0]


def case_reduce_init_order(rank, world, D):
    """fp64 partials whose sum depends on the order: with init the fold must
    start from it, ((init + p0) + p1) ... (reduce.hpp:81-83)."""
    part = torch.tensor([INIT_ORDER_VALS[rank % 4]], dtype=torch.float64)
    red = D.reduce_partials(part, "plus", init=-1e16).item()
    r, c, has = D.reduce_and_carry(part.clone(), "plus", init=-1e16)
    return red, r.item(), (c.item() if has else None), has


def case_gather_x_window(rank, world, D):
    """The windowed gemv exchange: every rank's window [lo, hi) of x, filled
    by one alltoallv, equals x[lo:hi] -- banded-like windows (own block +-
    a few columns), the whole x (random matrix), arbitrary windows; with
    x_local a view inside the window buffer (own part not sent) and apart."""
    n = 1003
    x = torch.arange(n, dtype=torch.float32) * 0.5 + 1
    segs = D.x_segments(n, world)
    s0, sl = segs[rank]
    out = []
    shapes = {
        "banded": lambda r: (max(0, segs[r][0] - 4), min(n, segs[r][0] + segs[r][1] + 5)),
        "random": lambda r: (0, n),
        "odd": lambda r: ((r * 131) % 400, min(n, (r * 131) % 400 + 300 + 97 * r)),
    }
    for name, f in shapes.items():
        lo, hi = f(rank)
        wins = D.x_windows(lo, hi, torch.device("cpu"))
        assert wins[rank] == (lo, hi)
        # apart
        xl = x[s0:s0 + sl].clone()
        xw = torch.full((hi - lo,), -1.0)
        D.gather_x_window(xl, xw, n, wins)
        out.append((name, "apart", bool(torch.equal(xw, x[lo:hi]))))
        # in place (own block inside the window buffer) when the window covers it
        if lo <= s0 and s0 + sl <= hi:
            xw2 = torch.full((hi - lo,), -1.0)
            xw2[s0 - lo:s0 - lo + sl].copy_(x[s0:s0 + sl])
            D.gather_x_window(xw2[s0 - lo:s0 - lo + sl], xw2, n, wins)
            out.append((name, "in_place", bool(torch.equal(xw2, x[lo:hi]))))
    return out


def case_reduce_and_carry(rank, world, D):
    """bench.py's N > 1 step: ONE all_gather of the segment partials gives the
    reduce result and this rank's scan carry (int32 wrapping, fp64, and a
    non-plus op through the fold loop)."""
    out = []
    for dt, vals in ((torch.int32, [2**31 - 5, 17, -9, 2**30]), (torch.float64, [0.1, 1e10, -3.5, 2.25])):
        v = vals[rank % len(vals)]
        r, c, has = D.reduce_and_carry(torch.tensor([v], dtype=dt), "plus")
        out.append((r.item(), c.item() if has else None, has))
    r, c, has = D.reduce_and_carry(torch.tensor([rank * 3 - 4], dtype=torch.int64), "max")
    out.append((r.item(), c.item() if has else None, has))
    return out


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

    allk = [np.random.default_rng(r + 10).integers(-50, 50, 5000 + 37 * r).astype(np.int32) for r in range(world)]
    out = D.dist_sort(keys, local_sort, samples_per_rank=64)
    return out.numpy(), np.concatenate(allk)


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

    allk = [np.random.default_rng(r + 10).integers(-50, 50, 5000 + 37 * r).astype(np.int32) for r in range(world)]
    out = D.dist_sort(keys, local_sort, merge_runs=merge_runs)
    assert seen == [True]
    return out.numpy(), np.concatenate(allk)


def case_sort_merge_into(rank, world, D):
    """dist_sort's copy-free destination step (bench.py, drhip_merge_runs_to):
    the all_to_all lands in `landing`, merge_into(src, dst, offsets) gets the
    runs there and must write the segment itself."""
    rng = np.random.default_rng(rank + 20)
    keys = torch.from_numpy(rng.integers(-500, 500, 4000 + 53 * rank).astype(np.int32))
    land = torch.full_like(keys, 12345)
    seen = []

    def local_sort(t):
        t.copy_(torch.from_numpy(np.sort(t.numpy())))

    def merge_into(src, dst, offs):
        assert src.data_ptr() == land.data_ptr() and dst.data_ptr() == keys.data_ptr()
        x = src.numpy()
        assert len(offs) == world + 1 and offs[0] == 0 and offs[-1] == x.size
        for a, b in zip(offs[:-1], offs[1:]):
            assert np.all(np.diff(x[a:b]) >= 0)
        seen.append(True)
        dst.copy_(torch.from_numpy(np.sort(x)))

    allk = [np.random.default_rng(r + 20).integers(-500, 500, 4000 + 53 * r).astype(np.int32) for r in range(world)]
    out = D.dist_sort(keys, local_sort, merge_into=merge_into, landing=land)
    assert seen == [True] and out.data_ptr() == keys.data_ptr()
    return out.numpy(), np.concatenate(allk)


def case_sort_float(rank, world, D):
    rng = np.random.default_rng(rank)
    keys = torch.from_numpy((rng.standard_normal(3000) * 100).astype(np.float32))
    _, to_bits, _ = D.key_bits(np.float32)

    def local_sort(t):
        t.copy_(torch.from_numpy(np.sort(t.numpy())))

    mine = keys.numpy().copy()
    out = D.dist_sort(keys, local_sort, samples_per_rank=100)
    return out.numpy(), mine


def _radix_sort_np(t, np_dt, D):
    """local_sort stand-in in the radix (bit) order the device sort uses."""
    _, to_bits, _ = D.key_bits(np_dt)
    x = t.numpy().view(np_dt)
    t.copy_(torch.from_numpy(x[np.argsort(to_bits(x), kind="stable")].view(t.numpy().dtype)))


SPLIT_SHAPES = {
    # name: (key dtype, per-rank sizes(world), key generator, samples per rank)
    "skewed": (np.uint32, lambda w: [20000 if r == 0 else 3 + r for r in range(w)],
               lambda g, n: g.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32), 32),
    "empty_rank": (np.int32, lambda w: [0 if r == 1 else 4000 + r for r in range(w)],
                   lambda g, n: g.integers(-3, 3, n).astype(np.int32), 16),
    "all_equal": (np.uint32, lambda w: [3000 + 11 * r for r in range(w)],
                  lambda g, n: np.full(n, 7, np.uint32), 8),
    "sorted_blocks": (np.int64, lambda w: [5000] * w,
                      lambda g, n: np.sort(g.integers(-(1 << 62), 1 << 62, n)).astype(np.int64), 8),
    "float64": (np.float64, lambda w: [2500 + 101 * r for r in range(w)],
                lambda g, n: (g.standard_normal(n) * 1e3).astype(np.float64), 50),
}


def case_sort_shapes(rank, world, D):
    """exact splitting over skewed sizes, an empty rank, all-equal keys,
    pre-sorted blocks (every boundary inside one rank) and 64-bit keys, with
    few samples per rank so the brackets hold many keys: every rank must end
    with its own key count and the concatenation must be the sorted input."""
    out = {}
    for name, (dt, sizes, gen, spr) in SPLIT_SHAPES.items():
        sz = sizes(world)
        allk = [gen(np.random.default_rng(1000 * r + 7), sz[r]) for r in range(world)]
        tdt = {np.uint32: torch.int32, np.int32: torch.int32, np.int64: torch.int64, np.float64: torch.float64}[dt]
        keys = torch.from_numpy(allk[rank].view({np.uint32: np.int32}.get(dt, dt)).copy()).to(tdt)
        got = D.dist_sort(keys, lambda t: _radix_sort_np(t, dt, D), key_dtype=dt, samples_per_rank=spr)
        out[name] = (got.numpy().view(dt).copy(), np.concatenate(allk))
    return out


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


def case_sort_collectives(rank, world, D):
    """Count the collectives one dist_sort issues: 2 allgathers (samples,
    boundary slices) and 1 all_to_all, nothing else."""
    calls = {}
    names = ["all_gather_into_tensor", "all_gather", "all_reduce", "all_to_all_single", "broadcast",
             "barrier", "batch_isend_irecv", "gather", "scatter"]
    saved = {k: getattr(dist, k) for k in names}

    def wrap(k):
        def f(*a, **kw):
            calls[k] = calls.get(k, 0) + 1
            return saved[k](*a, **kw)
        return f
    for k in names:
        setattr(dist, k, wrap(k))
    try:
        keys = torch.from_numpy(np.random.default_rng(rank).integers(0, 1000, 20000 + rank).astype(np.int32))
        D.dist_sort(keys, lambda t: t.copy_(torch.from_numpy(np.sort(t.numpy()))))
    finally:
        for k in names:
            setattr(dist, k, saved[k])
    return calls


CASES = {"bench_check_sort": case_bench_check_sort, "flag_slots": case_flag_slots,
         "flag_slots_open_failure": case_flag_slots_open_failure, "gather_x_window": case_gather_x_window, "reduce_init_order": case_reduce_init_order, "reduce_and_carry": case_reduce_and_carry,"sort_collectives": case_sort_collectives, "reduce": case_reduce, "halo_periodic": case_halo_periodic, "scan": case_scan, "sort": case_sort, "sort_merge": case_sort_merge, "sort_merge_into": case_sort_merge_into,
         "sort_float": case_sort_float, "sort_shapes": case_sort_shapes,
         "gather_x": case_gather_x, "halo": case_halo}


@pytest.mark.parametrize("world", [2, 3])
def test_reduce_partials(world):
    n = 1001
    ref = 5 + int((np.arange(n, dtype=np.int64) * 7 - 300).sum())
    assert run("reduce", world) == [ref] * world


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("via", ["", "@drhip"])
def test_gather_x_window(world, via):
    """gemv's x exchange restricted to each rank's column window (one
    alltoallv) -- torch.distributed and the drhip RCCL C-ABI arithmetic
    (emulated over gloo) -- equals the full replication on every column the
    rows read."""
    for rank_res in run("gather_x_window" + via, world):
        assert rank_res and all(ok for _, _, ok in rank_res), rank_res


@pytest.mark.parametrize("world", [2, 3])
def test_reduce_init_fold_order(world):
    """init seeds the left fold (advisor round 3): float results follow the
    reference's ((init op p0) op p1) order, and rank r's scan carry is init op
    p0 ... op p_{r-1} (init on piece 0 only, inclusive_scan.hpp:77-83)."""
    import functools
    p = [INIT_ORDER_VALS[r % 4] for r in range(world)]
    ref = functools.reduce(lambda a, b: a + b, p, -1e16)
    assert ref != -1e16 + functools.reduce(lambda a, b: a + b, p)  # the order matters here
    for r, (red, red2, carry, has) in enumerate(run("reduce_init_order", world)):
        assert red == ref and red2 == ref
        assert has and carry == functools.reduce(lambda a, b: a + b, p[:r], -1e16)


def test_reduce_init_fold_order_world1():
    """The same contract on one rank (advisor round 4): with init, rank 0's
    carry is init and has_carry is True at every world size, so a caller
    applies init once whether N is 1 or 8."""
    (red, red2, carry, has), = run("reduce_init_order", 1)
    assert red == red2 == INIT_ORDER_VALS[0] + -1e16
    assert has and carry == -1e16


@pytest.mark.parametrize("world", [2, 3])
def test_reduce_and_carry(world):
    res = run("reduce_and_carry", world)
    for dt_i, vals in enumerate(([2**31 - 5, 17, -9, 2**30], [0.1, 1e10, -3.5, 2.25])):
        v = [vals[r % len(vals)] for r in range(world)]
        if dt_i == 0:
            wrap = lambda a: (a + 2**31) % 2**32 - 2**31
            tot, pre = wrap(sum(v)), [wrap(sum(v[:r])) for r in range(world)]
        else:
            tot, pre = float(np.sum(v)), [float(np.sum(v[:r])) for r in range(world)]
        for r in range(world):
            got_r, got_c, has = res[r][dt_i]
            assert got_r == pytest.approx(tot, rel=1e-15) and has == (r > 0)
            if r:
                assert got_c == pytest.approx(pre[r], rel=1e-15)
    mx = [r * 3 - 4 for r in range(world)]
    for r in range(world):
        assert res[r][2] == (max(mx), max(mx[:r]) if r else None, r > 0)


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


@pytest.mark.parametrize("world", [2, 3])
def test_dist_sort_merge_into_landing(world):
    res = run("sort_merge_into", world)
    got = np.concatenate([r[0] for r in res])
    assert np.array_equal(got, np.sort(res[0][1]))
    for rank, r in enumerate(res):
        assert r[0].size == 4000 + 53 * rank


def test_dist_sort_float():
    res = run("sort_float", 2)
    got = np.concatenate([r[0] for r in res])
    assert np.array_equal(got, np.sort(np.concatenate([r[1] for r in res])))


@pytest.mark.parametrize("world", [2, 3, 4])
def test_dist_sort_split_shapes(world):
    res = run("sort_shapes", world)
    for name, (dt, sizes, _, _) in SPLIT_SHAPES.items():
        sz = sizes(world)
        got = np.concatenate([res[r][name][0] for r in range(world)])
        ref = res[0][name][1]
        _, to_bits, _ = __import__("dr_dist").key_bits(dt)
        assert np.array_equal(to_bits(got), np.sort(to_bits(ref))), name
        for r in range(world):
            assert res[r][name][0].size == sz[r], (name, r)


@pytest.mark.parametrize("world", [2, 3])
def test_dist_sort_collective_count(world):
    for calls in run("sort_collectives", world):
        assert calls == {"all_gather_into_tensor": 2, "all_to_all_single": 1}, calls


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


# ------------------------------------ the DrhipTransport (RCCL C-ABI) path
@pytest.mark.parametrize("world", [2, 3])
def test_drhip_transport_reduce_and_carry(world):
    a = run("reduce_and_carry", world)
    b = run("reduce_and_carry@drhip", world)
    assert a == b


@pytest.mark.parametrize("world", [2, 3, 4])
def test_drhip_transport_dist_sort(world):
    res = run("sort_shapes@drhip", world)
    for name, (dt, sizes, _, _) in SPLIT_SHAPES.items():
        sz = sizes(world)
        got = np.concatenate([res[r][name][0] for r in range(world)])
        _, to_bits, _ = __import__("dr_dist").key_bits(dt)
        assert np.array_equal(to_bits(got), np.sort(to_bits(res[0][name][1]))), name
        for r in range(world):
            assert res[r][name][0].size == sz[r], (name, r)


@pytest.mark.parametrize("world", [2, 3])
def test_drhip_transport_halo(world):
    for got, ref in run("halo@drhip", world):
        assert np.array_equal(got, ref)
    for got, want in run("halo_periodic@drhip", world):
        assert np.array_equal(got, want)


def test_drhip_transport_gather_x():
    for r in run("gather_x@drhip", 2):
        assert np.array_equal(r, np.array([0, 1, 2, 3, 10, 11, 12, 13], np.float32))


@pytest.mark.parametrize("world", [2, 3])
def test_bench_graph_phase_rank_symmetric_on_capture_failure(world):
    """bench.py c2_strong graph mode: a capture failure on rank 1 only
    (DRHIP_BENCH_FAIL_CAPTURE_RANK=1) makes EVERY rank report graph_error and
    skip the replays (no rank enters the captured collective alone), and
    the graph that did get captured is still destroyed."""
    res = run("bench_graph_phase:1", world)
    for r, (ms, err, nlaunch, destroyed) in enumerate(res):
        assert ms is None and nlaunch == 0
        if r == 1:
            assert err.startswith("capture: RuntimeError: injected") and destroyed == []
        else:
            assert "another rank" in err and destroyed == ["graph"]


def test_bench_graph_phase_all_ranks_ok():
    res = run("bench_graph_phase:none", 2)
    for ms, err, nlaunch, destroyed in res:
        assert ms == 1.5 and err is None and nlaunch == 5 and destroyed == ["graph"]


@pytest.mark.parametrize("world", [2, 3])
def test_flag_slots_bootstrap_and_gather(world):
    """dr_dist.FlagSlots (the bench's collective-free combine): every rank's
    slot array handle reaches every other rank, peers[] is in rank order
    with this rank's own array at its index, a 4- or 8-byte value per rank
    is gathered in rank order, and close() unmaps the peers and frees the
    local array."""
    res = run("flag_slots", world)
    for r, (peers, out, closed, freed) in enumerate(res):
        assert peers == [1000 + j for j in range(world)]
        assert out[0] == [0.5 + j for j in range(world)] and out[1] == [-7 * j for j in range(world)]
        assert sorted(closed) == [1000 + j for j in range(world) if j != r] and freed == [1000 + r]


@pytest.mark.parametrize("world", [2, 3])
def test_flag_slots_bootstrap_failure_unmaps(world):
    """A FlagSlots bootstrap whose last peer mapping fails raises on that
    rank after unmapping the peers it had mapped and freeing its own array
    (no IPC mapping or slot array leaks on the error path)."""
    res = run("flag_slots_open_failure", world)
    for r, (raised, closed, freed) in enumerate(res):
        last = max(j for j in range(world) if j != r)
        assert raised
        assert sorted(closed) == [1000 + j for j in range(world) if j not in (r, last)] and freed == [1000 + r]


@pytest.mark.parametrize("world", [2, 3])
def test_bench_sort_check_exact_at_n_gt_1(world):
    """The N > 1 sort check pins the exact sorted sequence: a correct output
    passes; a duplicated key (multiset changed) fails; two ranks' blocks
    swapped (each locally sorted, multiset intact) fail on the global ranks
    of their first / last keys."""
    res = run("bench_check_sort", world)
    for r, (good, dup, swapped) in enumerate(res):
        assert good is True and dup is False
        assert swapped["ok"] is False and swapped["multiset_hash_equal"] and swapped["locally_sorted"]
        if r < 2:
            assert not swapped["global_ranks_exact"]
