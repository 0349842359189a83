"""The flag-slot exchange (drhip_xchg_allgather, csrc/xchg.hip): the combine
of the strong-scaled reduce + inclusive_scan step without a collective
(SURVEY.md 5).  Parity:

  * w = 2 and 4 rank PROCESSES on one GPU (the one-rank-per-GPU bench's
    path), every slot array mapped into every process with drhip_ipc_handle
    / drhip_ipc_open: each rank posts its value, every rank gathers all w in
    rank order -- over repeated exchanges, so both epoch parities and the
    device-side exchange count are exercised, and again replayed from a HIP
    graph;
  * the strong-scaled C2 step on 4 rank processes (2^24 elements in total):
    drhip_reduce_tiles -> drhip_xchg_allgather -> drhip_inclusive_scan_tiles
    with the gathered partials: int32 bit-exact against the oracle's 3-phase
    scan (inclusive_scan.hpp:22-148), fp32 within 1e-5 of the fp64 prefix,
    and the reduce result (fold of all partials) equal on every rank.
Segments sharing a device inside ONE process are not exchange participants:
the HIP runtime multiplexes their streams onto a few hardware queues, so one
segment's waiting exchange kernel can sit ahead of another segment's post
(measured round 5: 8 duplicated segments hit the spin bound; the one-process
shp path folds pinned totals after event waits instead)."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _ipc_worker(rank, w, port, case, q):
    import traceback
    try:
        import torch
        import torch.distributed as dist
        import drhip as dr
        import oracle as O
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=w)
        dr.load()
        dr.init([0])
        local = dr.xchg_alloc(0, w)
        h = torch.frombuffer(bytearray(dr.ipc_handle(local)), dtype=torch.uint8)
        hs = [torch.empty_like(h) for _ in range(w)]
        dist.all_gather(hs, h)
        peers = [local if j == rank else dr.ipc_open(0, bytes(hs[j].numpy().tobytes())) for j in range(w)]
        bufs = []
        out = None
        if case == "gather":
            val = dr.DeviceArray(0, 1, np.uint64)
            gat = dr.DeviceArray(0, w, np.uint64)
            bufs = [val, gat]
            got = []
            for it in range(5):
                dr.h2d(0, val.ptr, np.array([1000 * it + rank + (rank << 40)], np.uint64))
                dr.xchg_allgather(0, local, peers, rank, val.ptr, gat.ptr)
                got.append(gat.numpy().tolist())
            dr.graph_begin(0)
            try:
                dr.xchg_allgather(0, local, peers, rank, val.ptr, gat.ptr)
            finally:
                ge = dr.graph_end(0)
            for it in range(3):
                dr.h2d(0, val.ptr, np.array([77 * it + rank], np.uint64))
                dr.graph_launch(0, ge)
                got.append(gat.numpy().tolist())
            dr.graph_destroy(ge)
            out = got
        else:  # "step_i32" / "step_f32": the strong-scaled C2 step
            dtype = np.int32 if case == "step_i32" else np.float32
            acc = np.int32 if dtype == np.int32 else np.float64
            n = 1 << 24
            rng = np.random.default_rng(5)
            x = rng.integers(0, 1 << 16, n, dtype=np.int32) if dtype == np.int32 else rng.random(n, dtype=np.float32)
            lens = O.dv_segments(n, w)
            off = sum(lens[:rank])
            m = lens[rank]
            src = dr.DeviceArray(0, m, dtype, host=x[off:off + m])
            dst = dr.DeviceArray(0, m, dtype)
            part, gat, res = dr.DeviceArray(0, 1, acc), dr.DeviceArray(0, w, acc), dr.DeviceArray(0, 1, acc)
            bufs = [src, dst, part, gat, res]
            outs = []
            for rep in range(2):
                dr.reduce_tiles_async(0, dtype, "plus", src.ptr, m, part.ptr)
                dr.xchg_allgather(0, local, peers, rank, part.ptr, gat.ptr, value_bytes=np.dtype(acc).itemsize)
                dr.scan_tiles_async(0, dtype, "plus", src.ptr, dst.ptr, m, partials=gat.ptr, w=w, rank=rank,
                                    result=res.ptr)
                y = dst.numpy()
                r = res.numpy()[0]
                if dtype == np.int32:
                    ok = bool(np.array_equal(y, O.shp_scan(x, lens, "plus")[off:off + m]))
                    rok = int(r) == int(O.shp_reduce(x, lens, 0))
                else:
                    ref = O.scan_exact_f32(x)[off:off + m]
                    ok = float(np.max(np.abs(y - ref) / np.maximum(np.abs(ref), 1e-30))) <= 1e-5
                    tot = O.reduce_exact(x)
                    rok = abs(float(r) - tot) <= 1e-5 * tot
                outs.append((ok, rok, float(r)))
            out = outs
        dr.sync(0)
        dist.barrier()
        for j in range(w):
            if j != rank:
                dr.ipc_close(0, peers[j])
        dist.barrier()
        for b in bufs:
            b.free()
        dr.xchg_free(0, local)
        dr.finalize()
        dist.destroy_process_group()
        q.put((rank, "ok", out))
    except Exception:  # noqa: BLE001 -- reported to the parent
        q.put((rank, "err", traceback.format_exc()))


def _run_ranks(w, case):
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ps = [ctx.Process(target=_ipc_worker, args=(r, w, port, case, q)) for r in range(w)]
    for p in ps:
        p.start()
    res = {}
    try:
        for _ in range(w):
            r, st, out = q.get(timeout=240)
            assert st == "ok", out
            res[r] = out
    finally:
        for p in ps:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    return [res[r] for r in range(w)]


@pytest.mark.parametrize("w", [2, 4])
def test_xchg_gather_rank_processes_ipc(w):
    res = _run_ranks(w, "gather")
    want = [[1000 * it + j + (j << 40) for j in range(w)] for it in range(5)]
    want += [[77 * it + j for j in range(w)] for it in range(3)]
    for r in range(w):
        assert res[r] == want, r


@pytest.mark.parametrize("dtype", ["i32", "f32"])
def test_xchg_strong_step_rank_processes(dtype):
    res = _run_ranks(4, "step_" + dtype)
    for r, outs in enumerate(res):
        for ok, rok, _ in outs:
            assert ok and rok, (r, outs)
    # every rank folded the same gathered partials into the same reduce result
    assert len({outs[0][2] for outs in res}) == 1
