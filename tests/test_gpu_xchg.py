"""The flag-slot exchange (drhip_xchg_allgather, csrc/xchg.hip): the combine
of the strong-scaled reduce + inclusive_scan step without a collective
(SURVEY.md 5).  Parity:

  * 8 segments duplicated on one GPU, one process (every slot array reached
    through plain device pointers): each segment posts its value, every
    segment gathers all 8 in rank order -- over repeated exchanges, so both
    epoch parities and the device-side exchange count are exercised, also
    when the exchange is replayed from a HIP graph;
  * the strong-scaled C2 step on those 8 segments (2^24 elements in total):
    drhip_reduce_tiles -> drhip_xchg_allgather -> drhip_inclusive_scan_tiles
    with the gathered partials: int32 bit-exact against the oracle's 3-phase
    scan (inclusive_scan.hpp:22-148), fp32 within 1e-5 of the fp64 prefix,
    and the reduce result (fold of all partials) equal on every segment;
  * two PROCESSES on one GPU, the slot arrays mapped across them with
    drhip_ipc_handle / drhip_ipc_open (the one-rank-per-GPU bench's path):
    the same gather, so IPC is known to work before bench.py relies on it."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _reinit(dr, devs):
    dr.finalize()
    dr.init(devs)


def test_xchg_eight_segments_repeated_and_graph(dr):
    P = 8
    _reinit(dr, [0] * P)
    slots = [dr.xchg_alloc(k, P) for k in range(P)]
    vals = [dr.DeviceArray(k, 1, np.uint64) for k in range(P)]
    outs = [dr.DeviceArray(k, P, np.uint64) for k in range(P)]
    graphs = []
    try:
        for it in range(5):
            want = np.array([(it + 1) * 1000 + k * 7 + (k << 40) for k in range(P)], np.uint64)
            for k in range(P):
                dr.h2d(k, vals[k].ptr, want[k:k + 1])
            for k in range(P):
                dr.xchg_allgather(k, slots[k], slots, k, vals[k].ptr, outs[k].ptr)
            dr.sync()
            for k in range(P):
                assert np.array_equal(outs[k].numpy(), want), (it, k)
        # the exchange captured once per segment and replayed: the epoch is
        # counted on the device, so every replay is a new exchange
        for k in range(P):
            dr.graph_begin(k)
            try:
                dr.xchg_allgather(k, slots[k], slots, k, vals[k].ptr, outs[k].ptr)
            finally:
                graphs.append(dr.graph_end(k))
        for it in range(3):
            want = np.array([it * 31 + k for k in range(P)], np.uint64)
            for k in range(P):
                dr.h2d(k, vals[k].ptr, want[k:k + 1])
            for k in range(P):
                dr.graph_launch(k, graphs[k])
            dr.sync()
            for k in range(P):
                assert np.array_equal(outs[k].numpy(), want), ("graph", it, k)
    finally:
        for g in graphs:
            dr.graph_destroy(g)
        for b in vals + outs:
            b.free()
        for k in range(P):
            dr.xchg_free(k, slots[k])
        _reinit(dr, [0])


@pytest.mark.parametrize("dtype", [np.int32, np.float32])
def test_xchg_strong_step_eight_segments(dr, oracle, dtype):
    P, n = 8, 1 << 24
    rng = np.random.default_rng(5)
    x = rng.integers(0, 1 << 16, n, dtype=np.int32) if dtype == np.int32 else rng.random(n, dtype=np.float32)
    acc = np.int32 if dtype == np.int32 else np.float64
    lens = oracle.dv_segments(n, P)
    _reinit(dr, [0] * P)
    slots = [dr.xchg_alloc(k, P) for k in range(P)]
    bufs = []
    try:
        off = 0
        for k in range(P):
            src = dr.DeviceArray(k, lens[k], dtype, host=x[off:off + lens[k]])
            dst = dr.DeviceArray(k, lens[k], dtype)
            part = dr.DeviceArray(k, 1, acc)
            gat = dr.DeviceArray(k, P, acc)
            res = dr.DeviceArray(k, 1, acc)
            bufs.append((src, dst, part, gat, res))
            off += lens[k]
        vb = np.dtype(acc).itemsize
        for rep in range(2):
            for k, (src, dst, part, gat, res) in enumerate(bufs):
                dr.reduce_tiles_async(k, dtype, "plus", src.ptr, lens[k], part.ptr)
                dr.xchg_allgather(k, slots[k], slots, k, part.ptr, gat.ptr, value_bytes=vb)
                dr.scan_tiles_async(k, dtype, "plus", src.ptr, dst.ptr, lens[k], partials=gat.ptr, w=P, rank=k,
                                    result=res.ptr)
            dr.sync()
            got = np.concatenate([b[1].numpy() for b in bufs])
            results = [b[4].numpy()[0] for b in bufs]
            if dtype == np.int32:
                assert np.array_equal(got, oracle.shp_scan(x, lens, "plus"))
                assert all(int(r) == int(oracle.shp_reduce(x, lens, 0)) for r in results)
            else:
                ref = oracle.scan_exact_f32(x)
                assert float(np.max(np.abs(got - ref) / np.maximum(np.abs(ref), 1e-30))) <= 1e-5
                tot = oracle.reduce_exact(x)
                assert all(abs(float(r) - tot) <= 1e-5 * tot for r in results)
                assert len(set(float(r) for r in results)) == 1  # every segment folds the same partials
    finally:
        for b in bufs:
            for a in b:
                a.free()
        for k in range(P):
            dr.xchg_free(k, slots[k])
        _reinit(dr, [0])


def _ipc_worker(rank, w, port, q):
    import traceback
    try:
        import torch
        import torch.distributed as dist
        import drhip as dr
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
        val = dr.DeviceArray(0, 1, np.uint64)
        out = dr.DeviceArray(0, w, np.uint64)
        got = []
        for it in range(4):
            dr.h2d(0, val.ptr, np.array([1000 * it + rank], np.uint64))
            dr.xchg_allgather(0, local, peers, rank, val.ptr, out.ptr)
            got.append(out.numpy().tolist())
        dist.barrier()
        for j in range(w):
            if j != rank:
                dr.ipc_close(0, peers[j])
        dist.barrier()
        val.free()
        out.free()
        dr.xchg_free(0, local)
        dr.finalize()
        dist.destroy_process_group()
        q.put((rank, "ok", got))
    except Exception:  # noqa: BLE001 -- reported to the parent
        q.put((rank, "err", traceback.format_exc()))


def test_xchg_two_processes_ipc_one_gpu():
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    w = 2
    ps = [ctx.Process(target=_ipc_worker, args=(r, w, port, q)) for r in range(w)]
    for p in ps:
        p.start()
    res = {}
    try:
        for _ in range(w):
            r, st, out = q.get(timeout=180)
            assert st == "ok", out
            res[r] = out
    finally:
        for p in ps:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for r in range(w):
        assert res[r] == [[1000 * it + j for j in range(w)] for it in range(4)]
