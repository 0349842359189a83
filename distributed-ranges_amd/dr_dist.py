"""Multi-process (one rank per GPU) combine steps of the shp algorithms.

The reference's shp layer is one process driving many devices; for the
per-GPU-process benchmark (and any multi-node use) the cross-segment steps
become collectives over torch.distributed ("nccl" = RCCL over xGMI on the
GPU box, "gloo" in the CPU tests).  Each function takes the rank's local
compute as callables (`ops`), so the same host logic is exercised by the
world_size-2 gloo tests with numpy kernels and by bench.py with the
libdrhip kernels.

  reduce    shp/algorithms/reduce.hpp:81-83   fold of per-segment partials in
                                              segment order
  scan      inclusive_scan.hpp:103-143        carry = exclusive prefix of the
                                              preceding segments' totals
  sort      (new)              samples + slices allgathers,
                                              exact splitting, all-to-all
  gemv      gemv.hpp:30-42                    x: every rank receives the
                                              window of x its rows' columns
                                              span (alltoallv; the whole x
                                              only for a random matrix)
  halo      details/halo.hpp:336-387          r cells to rank-1 / rank+1
"""
import numpy as np
import torch
import torch.distributed as dist

OPS = {
    "plus": lambda a, b: a + b,
    "mul": lambda a, b: a * b,
    "min": lambda a, b: torch.minimum(a, b),
    "max": lambda a, b: torch.maximum(a, b),
}


class TorchTransport:
    """The three exchanges of the shp combine steps over torch.distributed:
    the world_size-2/3 `gloo` CPU tests (and the one-GPU rehearsal of the
    N > 1 bench); gloo cannot run these collectives on device tensors, so
    device tensors are staged through host memory there."""

    name = "torch.distributed"

    def world(self):
        return (dist.get_world_size(), dist.get_rank()) if dist.is_initialized() else (1, 0)

    def _staged(self, t):
        return dist.get_backend() == "gloo" and t.is_cuda

    def all_gather_into(self, out, inp):
        """out = the w equal blocks `inp` of every rank, in rank order."""
        if self._staged(inp):
            o = out.cpu()
            dist.all_gather_into_tensor(o, inp.cpu())
            out.copy_(o)
        else:
            dist.all_gather_into_tensor(out, inp)

    def all_to_all(self, out, inp, recv_counts, send_counts):
        """elements inp[send_off[j] : + send_counts[j]] -> rank j; out holds
        the received blocks in rank order."""
        if self._staged(inp):
            src, o = inp.cpu(), out.cpu()
            dist.all_to_all_single(o, src, output_split_sizes=recv_counts, input_split_sizes=send_counts)
            out.copy_(o)
        else:
            dist.all_to_all_single(out, inp, output_split_sizes=recv_counts, input_split_sizes=send_counts)

    def alltoallv(self, out, recv_counts, recv_offs, inp, send_counts, send_offs):
        """elements inp[send_offs[j] : + send_counts[j]] -> rank j, landing at
        out[recv_offs[i] : + recv_counts[i]] of rank j for source i; pieces
        may overlap on the send side (grouped point-to-point)."""
        w, r = self.world()
        dev = torch.device("cpu") if self._staged(inp) else inp.device
        ops, land = [], []
        for j in range(w):
            if j == r:
                if send_counts[j]:
                    a, b = int(send_offs[j]), int(recv_offs[j])
                    out[b:b + int(recv_counts[j])].copy_(inp[a:a + int(send_counts[j])])
                continue
            if send_counts[j]:
                a = int(send_offs[j])
                ops.append(dist.P2POp(dist.isend, inp[a:a + int(send_counts[j])].to(dev).contiguous(), j))
            if recv_counts[j]:
                t = torch.empty(int(recv_counts[j]), dtype=out.dtype, device=dev)
                ops.append(dist.P2POp(dist.irecv, t, j))
                land.append((int(recv_offs[j]), t))
        for q in (dist.batch_isend_irecv(ops) if ops else []):
            q.wait()
        for b, t in land:
            out[b:b + t.numel()].copy_(t)

    def halo(self, buf, radius, periodic):
        """span_halo exchange of a [radius | owned | radius] buffer (w > 1)."""
        w, r = self.world()
        dev = torch.device("cpu") if self._staged(buf) else buf.device
        n_owned = buf.numel() - 2 * radius
        do_prev, do_next = periodic or r > 0, periodic or r < w - 1
        rprev, rnext = (r - 1) % w, (r + 1) % w
        ops = []
        if do_prev:
            ops.append(dist.P2POp(dist.isend, buf[radius:2 * radius].to(dev).contiguous(), rprev))
        if do_next:
            ops.append(dist.P2POp(dist.isend, buf[n_owned:n_owned + radius].to(dev).contiguous(), rnext))
            hi_halo = torch.empty(radius, dtype=buf.dtype, device=dev)
            ops.append(dist.P2POp(dist.irecv, hi_halo, rnext))
        if do_prev:
            lo_halo = torch.empty(radius, dtype=buf.dtype, device=dev)
            ops.append(dist.P2POp(dist.irecv, lo_halo, rprev))
        for q in dist.batch_isend_irecv(ops):
            q.wait()
        if do_prev:
            buf[:radius].copy_(lo_halo)
        if do_next:
            buf[n_owned + radius:].copy_(hi_halo)


class FlagSlots:
    """The combine of a strong-scaled reduce + scan step without a
    collective (drhip_xchg_allgather, csrc/xchg.hip): every rank's slot array
    (fine-grained device memory) mapped into every other rank's process with
    drhip_ipc_handle / drhip_ipc_open; the handles travel once over the
    torch.distributed group `group` (the host-side gloo group in bench.py).
    all_gather_into(out, inp) gathers one 4- or 8-byte device value per
    rank into out[0..w) in rank order, on segment `seg`'s stream -- the
    same contract as DrhipTransport.all_gather_into for a 1-element inp.
    `lib` is the drhip module."""

    name = "drhip flag slots (IPC-mapped, no collective)"

    def __init__(self, seg, local, peers, rank, lib):
        self.seg, self.local, self.peers, self.rank, self.lib = seg, local, peers, rank, lib
        self.opened = [p for j, p in enumerate(peers) if j != rank]

    @classmethod
    def bootstrap(cls, seg=0, lib=None, group=None):
        if lib is None:
            import drhip as lib
        w, r = dist.get_world_size(group), dist.get_rank(group)
        local = lib.xchg_alloc(seg, w)
        opened = []
        try:
            handles = [None] * w
            dist.all_gather_object(handles, lib.ipc_handle(local), group=group)
            peers = []
            for j in range(w):
                if j == r:
                    peers.append(local)
                else:
                    peers.append(lib.ipc_open(seg, handles[j]))
                    opened.append(peers[-1])
        except Exception:
            for p in opened:  # a failure part-way: unmap what was mapped
                try:
                    lib.ipc_close(seg, p)
                except Exception:  # noqa: BLE001 -- the first error is the one raised
                    pass
            lib.xchg_free(seg, local)
            raise
        return cls(seg, local, peers, r, lib)

    def all_gather_into(self, out, inp):
        assert out.numel() == len(self.peers) and inp.numel() == 1 and out.dtype == inp.dtype
        assert inp.element_size() in (4, 8)
        self.lib.xchg_allgather(self.seg, self.local, self.peers, self.rank, inp.data_ptr(), out.data_ptr(),
                                value_bytes=inp.element_size())

    def close(self):
        for p in self.opened:
            self.lib.ipc_close(self.seg, p)
        self.opened = []
        if self.local:
            self.lib.xchg_free(self.seg, self.local)
            self.local = None


class DrhipTransport:
    """The same exchanges through libdrhip's own RCCL C-ABI (csrc/comm.hip:
    drhip_allgather, drhip_alltoallv, drhip_halo_exchange), enqueued on
    segment `seg`'s stream: the product path of the one-process-per-GPU mode
    (bench.py at N > 1).  torch.distributed only bootstraps it: rank 0's
    drhip_comm_unique_id travels over the process group's store, then every
    rank calls drhip_comm_init_rank.  Device tensors only.  Work the caller
    queued on torch's current stream is ordered before each exchange, and
    the exchange before later work on that stream (no-ops when the caller
    already runs on the segment stream, as bench.py does).
    `lib` is the drhip module (a CPU test passes an emulation of the four
    calls over gloo to check this class's byte/offset arithmetic)."""

    name = "drhip RCCL C-ABI"

    def __init__(self, seg=0, lib=None, stream=None):
        if lib is None:
            import drhip as lib
        self.lib, self.seg = lib, seg
        self.stream = stream
        self._w = lib.comm_rank(seg)[::-1]  # (nranks, rank)

    @classmethod
    def bootstrap(cls, seg=0, lib=None, stream=None):
        """rank 0 makes the RCCL unique id, the torch.distributed store
        carries it, every rank joins (drhip_comm_init_rank)."""
        if lib is None:
            import drhip as lib
        w, r = dist.get_world_size(), dist.get_rank()
        obj = [lib.comm_unique_id() if r == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        lib.comm_init_rank(seg, w, r, obj[0])
        return cls(seg, lib, stream)

    def world(self):
        return self._w

    def _fence_in(self):
        if self.stream is not None and torch.cuda.is_available():
            cur = torch.cuda.current_stream()
            if cur.cuda_stream != self.stream.cuda_stream:
                self.stream.wait_stream(cur)
                return cur
        return None

    def _fence_out(self, cur):
        if cur is not None:
            cur.wait_stream(self.stream)

    def all_gather_into(self, out, inp):
        inp = inp.contiguous()
        assert out.numel() == self._w[0] * inp.numel() and out.dtype == inp.dtype
        cur = self._fence_in()
        self.lib.allgather(self.seg, inp.data_ptr(), out.data_ptr(), inp.numel() * inp.element_size())
        self._fence_out(cur)

    def all_to_all(self, out, inp, recv_counts, send_counts):
        inp = inp.contiguous()
        esz = inp.element_size()
        sb = np.asarray(send_counts, np.uint64) * esz
        rb = np.asarray(recv_counts, np.uint64) * esz
        so = np.concatenate([[0], np.cumsum(sb)[:-1]]).astype(np.uint64)
        ro = np.concatenate([[0], np.cumsum(rb)[:-1]]).astype(np.uint64)
        cur = self._fence_in()
        self.lib.alltoallv(self.seg, inp.data_ptr(), sb, so, out.data_ptr(), rb, ro)
        self._fence_out(cur)

    def alltoallv(self, out, recv_counts, recv_offs, inp, send_counts, send_offs):
        esz = inp.element_size()
        assert out.is_contiguous() and inp.is_contiguous() and out.dtype == inp.dtype
        b = [np.asarray(v, np.uint64) * esz for v in (send_counts, send_offs, recv_counts, recv_offs)]
        cur = self._fence_in()
        self.lib.alltoallv(self.seg, inp.data_ptr(), b[0], b[1], out.data_ptr(), b[2], b[3])
        self._fence_out(cur)

    def halo(self, buf, radius, periodic):
        assert buf.is_contiguous()
        cur = self._fence_in()
        self.lib.halo_exchange(self.seg, buf.data_ptr(), buf.numel() - 2 * radius, buf.element_size(), radius,
                               radius, periodic)
        self._fence_out(cur)


_transport = TorchTransport()


def use(transport):
    """Select the transport of every combine step below (TorchTransport by
    default; bench.py selects DrhipTransport on the GPU box at N > 1).
    Returns the previous one."""
    global _transport
    prev, _transport = _transport, transport
    return prev


def transport():
    return _transport


def world():
    return _transport.world()


def _all_gather_into(out, inp):
    _transport.all_gather_into(out, inp)


def reduce_partials(partial, op="plus", init=None):
    """partial: 1-element tensor (the rank's segment result, ACC type).
    Returns the fold init op p_0 op p_1 ... in rank (= segment) order, on
    every rank (reduce.hpp:81-83)."""
    w, r = world()
    if w == 1:
        return partial.clone() if init is None else OPS[op](torch.full_like(partial, init), partial)
    g = torch.empty(w, dtype=partial.dtype, device=partial.device)
    _all_gather_into(g, partial.reshape(1))
    acc, _ = _fold(_seeded(g, init), op, r)
    return acc


def _seeded(g, init):
    """g, or [init, g...] so that the left fold starts from init: the
    reference's order ((init op p0) op p1) ... (reduce.hpp:81-83), which
    for floats differs from init op (p0 op p1 ...)."""
    if init is None:
        return g
    return torch.cat([torch.full((1,), init, dtype=g.dtype, device=g.device), g])


def _fold(g, op, rank):
    """(fold of all w gathered partials, fold of those of ranks < rank or
    None) -- left folds in segment order (reduce.hpp:81-83,
    inclusive_scan.hpp:108-116).  Device tensors: ONE drhip_fold_partials
    kernel (a single thread folds the w values in order, so float partials
    fold exactly as the reference's host loop); host tensors: the same loop
    in torch ops."""
    w = g.numel()
    if g.is_cuda:
        import drhip
        seg = getattr(_transport, "seg", 0)
        res = torch.empty(1, dtype=g.dtype, device=g.device)
        carry = torch.empty(1, dtype=g.dtype, device=g.device)
        cur = torch.cuda.current_stream()
        ext = None
        if cur.cuda_stream != drhip.stream(seg):  # order the kernel between the caller's stream's work
            ext = torch.cuda.ExternalStream(drhip.stream(seg))
            ext.wait_stream(cur)
        drhip.fold_partials_async(seg, g.dtype, op, g.data_ptr(), w, rank, res.data_ptr(), carry.data_ptr())
        if ext is not None:
            cur.wait_stream(ext)
        return res, (carry if rank > 0 else None)
    acc = g[0:1].clone()
    carry = None
    for k in range(1, w):
        if k == rank:
            carry = acc.clone()
        acc = OPS[op](acc, g[k:k + 1])
    return acc, carry


def gather_partials(partial, out):
    """out[w] = every rank's 1-element partial, in rank (= segment) order:
    the one exchange of a reduce + scan step (the scan kernel then folds
    them itself, drhip_inclusive_scan_gathered)."""
    w, _ = world()
    if w == 1:
        out.copy_(partial.reshape(1))
        return out
    _all_gather_into(out, partial.reshape(1))
    return out


def scan_carry(total, op="plus"):
    """total: 1-element tensor (the rank's segment total, ACC type).  Returns
    (carry, has_carry): the op-fold of the totals of ranks < this rank, as a
    1-element tensor on the same device (read by the scan kernel as
    carry_dev), and whether one exists (rank 0 has none)."""
    w, r = world()
    if w == 1:
        return None, False
    g = torch.empty(w, dtype=total.dtype, device=total.device)
    _all_gather_into(g, total.reshape(1))
    if r == 0:
        return None, False
    _, carry = _fold(g, op, r)
    return carry, True


def reduce_and_carry(partial, op="plus", init=None):
    """One all_gather of the segment results serving both shp::reduce and
    the carry of shp::inclusive_scan over the same range (a reduce + scan
    step, bench.py): returns (result, carry, has_carry) -- the fold of all
    partials in segment order (reduce.hpp:81-83) and the fold of the
    partials of ranks < this rank (inclusive_scan.hpp:108-116).  With init,
    both folds start from it (init applies to piece 0 only, :77-83): the
    result is ((init op p0) op p1) ..., rank r's carry init op p0 ... op
    p_{r-1} (rank 0's carry is init)."""
    w, r = world()
    if w == 1:
        if init is None:
            return partial.clone(), None, False
        # as at w > 1: rank 0's carry is init (a caller must not apply init
        # again), whatever the world size
        seed = torch.full_like(partial, init)
        return OPS[op](seed, partial), seed, True
    g = torch.empty(w, dtype=partial.dtype, device=partial.device)
    _all_gather_into(g, partial.reshape(1))
    # both folds from the one gather (on the device: one kernel)
    acc, carry = _fold(_seeded(g, init), op, r if init is None else r + 1)
    return acc, carry, carry is not None


# ------------------------------------------------------------------ sort

def key_bits(dtype):
    """(unsigned numpy dtype, to_bits(ndarray), from_bits(ndarray)) of the
    radix order: order-preserving unsigned images of the keys."""
    dt = np.dtype(dtype)
    if dt == np.uint32:
        return np.uint32, (lambda x: x.view(np.uint32)), (lambda u: u.view(np.uint32))
    if dt == np.int32:
        return (np.uint32, lambda x: x.view(np.uint32) ^ np.uint32(0x80000000),
                lambda u: (u ^ np.uint32(0x80000000)).view(np.int32))
    if dt == np.float32:
        def tb(x):
            u = x.view(np.uint32)
            return u ^ np.where(u & np.uint32(0x80000000), np.uint32(0xFFFFFFFF), np.uint32(0x80000000))

        def fb(u):
            u = np.asarray(u, np.uint32)
            v = u ^ np.where(u & np.uint32(0x80000000), np.uint32(0x80000000), np.uint32(0xFFFFFFFF))
            return v.astype(np.uint32).view(np.float32)
        return np.uint32, tb, fb
    if dt == np.uint64:
        return np.uint64, (lambda x: x.view(np.uint64)), (lambda u: u.view(np.uint64))
    if dt == np.int64:
        return (np.uint64, lambda x: x.view(np.uint64) ^ np.uint64(1 << 63),
                lambda u: (np.asarray(u, np.uint64) ^ np.uint64(1 << 63)).view(np.int64))
    if dt == np.float64:
        def tb64(x):
            u = x.view(np.uint64)
            return u ^ np.where(u & np.uint64(1 << 63), np.uint64(0xFFFFFFFFFFFFFFFF), np.uint64(1 << 63))

        def fb64(u):
            u = np.asarray(u, np.uint64)
            return (u ^ np.where(u & np.uint64(1 << 63), np.uint64(1 << 63),
                                 np.uint64(0xFFFFFFFFFFFFFFFF))).view(np.float64)
        return np.uint64, tb64, fb64
    raise TypeError(f"dist sort: unsupported key type {dt}")


SAMPLES_PER_RANK = 1 << 16


def _bytes_of(t):
    return t.contiguous().view(torch.uint8).reshape(-1)


def _gather_bytes(buf):
    """all_gather of equal-length uint8 tensors -> host ndarray [w, len]."""
    w, _ = world()
    out = torch.empty(w * buf.numel(), dtype=torch.uint8, device=buf.device)
    _all_gather_into(out, buf)
    return out.cpu().numpy().reshape(w, -1)


def exact_splits(keys, np_dt, samples_per_rank=SAMPLES_PER_RANK):
    """Exact splitting of the globally sorted order at the rank boundaries
    (every rank keeps its key count), from two allgathers:

      1. n, a stride t and the regular samples keys[::t] of every rank;
      2. every rank's slices of its sorted keys that hold the key of each
         boundary's global rank (drhip_split_windows brackets it from the
         samples; csrc/split.hip states the bounds);
    then drhip_split_exact finds each boundary key on the merged slices and
    splits ties in rank order -- the same host code shp::sort runs in one
    process.  keys: this rank's sorted keys (1-D tensor, np_dt keys).
    Returns (send_counts[w], recv_counts[w]) for all_to_all_single."""
    import drhip
    w, r = world()
    n = keys.numel()
    if w == 1:
        return [n], [n]
    _, to_bits, _ = key_bits(np_dt)
    isz = np.dtype(np_dt).itemsize
    t = max(1, -(-n // samples_per_rank))
    ns = -(-n // t)
    hdr = torch.tensor([n, t, ns], dtype=torch.int64).view(torch.uint8)
    buf = torch.zeros(24 + samples_per_rank * isz, dtype=torch.uint8, device=keys.device)
    buf[:24].copy_(hdr)
    if ns:
        buf[24:24 + ns * isz].copy_(_bytes_of(keys[::t]))
    host = _gather_bytes(buf)                                     # collective 1
    hd = np.stack([host[i, :24].view(np.int64) for i in range(w)]).astype(np.uint64)
    nn, tt, nsm = hd[:, 0], hd[:, 1], hd[:, 2]
    smp = np.concatenate([to_bits(host[i, 24:24 + int(nsm[i]) * isz].view(np_dt)).astype(np.uint64)
                          for i in range(w)])
    g = np.cumsum(nn)[:w - 1].astype(np.uint64)
    lo, hi, win = drhip.split_windows(nn, tt, nsm, smp, g)
    lens = (win[:, :, 1] - win[:, :, 0]).sum(axis=1).astype(np.int64)  # slice keys per rank
    lmax = int(lens.max())
    buf2 = torch.zeros(max(lmax, 1) * isz, dtype=torch.uint8, device=keys.device)
    if lens[r]:
        mine = torch.cat([keys[int(a):int(b)] for a, b in win[r]])
        buf2[:lens[r] * isz].copy_(_bytes_of(mine))
    host2 = _gather_bytes(buf2)                                   # collective 2
    wk = np.concatenate([to_bits(host2[i, :lens[i] * isz].view(np_dt)).astype(np.uint64) for i in range(w)])
    split = drhip.split_exact(nn, g, lo, hi, win, wk).astype(np.int64)
    prev = np.concatenate([np.zeros((w, 1), np.int64), split[:, :w - 1]], axis=1)
    send = (split[r] - prev[r]).tolist()
    recv = (split[:, r] - prev[:, r]).tolist()
    return send, recv


def dist_sort(keys, local_sort, key_dtype=None, merge_runs=None, samples_per_rank=SAMPLES_PER_RANK,
              merge_into=None, landing=None):
    """Sort the distributed range whose local segment is `keys` (a 1-D
    tensor, modified in place: every rank keeps its key count).
    local_sort(t): sorts t in place on its device (radix order).
    key_dtype: numpy key type when the tensor carries other bits (uint32
    keys in an int32 tensor).
    merge_into(src, dst, offsets): the destination step -- dst = the merge
    of src's sorted runs (one per source rank, offsets 0 .. n); the
    all_to_all lands in `landing` (a buffer like keys, allocated when None)
    and the merge writes straight into keys: no key copy before or after.
    merge_runs(t, offsets) (older form): sorts t in place; the received
    runs are first copied into keys.  Without either, a second local_sort.
    Collectives: 2 small allgathers (exact_splits) + 1 all_to_all."""
    local_sort(keys)
    w, _ = world()
    if w == 1:
        return keys
    np_dt = key_dtype or {torch.int32: np.int32, torch.float32: np.float32,
                          torch.int64: np.int64, torch.float64: np.float64}[keys.dtype]
    send, recv = exact_splits(keys, np_dt, samples_per_rank)
    out = landing if landing is not None else torch.empty_like(keys)
    _transport.all_to_all(out, keys, recv, send)
    offs = np.concatenate([[0], np.cumsum(recv)]).astype(np.int64)
    if merge_into is not None:
        merge_into(out, keys, offs)
        return keys
    keys.copy_(out)
    if merge_runs is not None:
        merge_runs(keys, offs)
    else:
        local_sort(keys)
    return keys


# ------------------------------------------------------------------ gemv

def gather_x(x_local):
    """gemv.hpp:30-42: every rank receives the whole b (all_gather of equal
    segments)."""
    w, _ = world()
    if w == 1:
        return x_local
    full = torch.empty(w * x_local.numel(), dtype=x_local.dtype, device=x_local.device)
    _all_gather_into(full, x_local)
    return full


def x_segments(n, w):
    """(start, length) of every rank's block of x (ceil(n/w) per rank,
    shp/distributed_vector.hpp:142)."""
    s = -(-n // w)
    return [(min(n, r * s), max(0, min(n, (r + 1) * s) - min(n, r * s))) for r in range(w)]


def x_windows(lo, hi, device):
    """Every rank's column window [lo, hi) of x -- recorded once, at matrix
    construction, by one all_gather (the tile's min and max column)."""
    w, _ = world()
    mine = torch.tensor([lo, hi], dtype=torch.int64, device=device)
    if w == 1:
        return [(lo, hi)]
    allw = torch.empty(2 * w, dtype=torch.int64, device=device)
    _all_gather_into(allw, mine)
    v = allw.cpu().tolist()
    return [(v[2 * i], v[2 * i + 1]) for i in range(w)]


def window_plan(n, windows, rank):
    """Element counts / offsets of the windowed x exchange for `rank`:
    send to i the part of this rank's x block inside i's window (offsets
    from the block's start); receive from j the part of j's block inside
    this rank's window (offsets from the window's start)."""
    w = len(windows)
    segs = x_segments(n, w)
    s0, sl = segs[rank]
    lo_me, hi_me = windows[rank]
    sc, so, rc, ro = [0] * w, [0] * w, [0] * w, [0] * w
    for i in range(w):
        a, b = max(s0, windows[i][0]), min(s0 + sl, windows[i][1])
        if a < b:
            sc[i], so[i] = b - a, a - s0
        j0, jl = segs[i]
        a, b = max(j0, lo_me), min(j0 + jl, hi_me)
        if a < b:
            rc[i], ro[i] = b - a, a - lo_me
    return sc, so, rc, ro


def gather_x_window(x_local, xw, n, windows, plan=None):
    """The gemv exchange restricted to the columns each rank's rows read:
    xw (this rank's window [lo, hi) of x) receives, from every rank, the part
    of its x block inside the window -- ONE alltoallv; for a banded matrix
    that is the rank's own block plus +-5 neighbour elements, for a random
    matrix all of x (then the same bytes as gather_x).  When x_local already
    sits inside xw at its place (a view), the rank's own part is not sent.
    The result at every column the rows read equals gather_x's."""
    w, r = world()
    sc, so, rc, ro = plan or window_plan(n, windows, r)
    lo = windows[r][0]
    s0 = x_segments(n, w)[r][0]
    esz = xw.element_size()
    in_place = x_local.numel() and rc[r] and x_local.data_ptr() == xw.data_ptr() + (s0 - lo) * esz
    if in_place:
        sc, rc = list(sc), list(rc)
        sc[r] = rc[r] = 0
    if w == 1:
        if rc[0]:
            xw[ro[0]:ro[0] + rc[0]].copy_(x_local[so[0]:so[0] + sc[0]])
        return xw
    _transport.alltoallv(xw, rc, ro, x_local, sc, so)
    return xw


# ------------------------------------------------------------------ halo

def halo_exchange(buf, radius, periodic=False):
    """1-D span_halo exchange (details/halo.hpp:336-387) on a buffer laid out
    [r halo | owned | r halo]: the first r owned cells go to rank-1 (tag
    halo_reverse), the last r owned cells to rank+1 (halo_forward); the ends
    keep their halos unless periodic.  Sends are issued [reverse, forward]
    and receives [next halo, prev halo] -- the order csrc/comm.hip's
    drhip_halo_exchange uses with RCCL, which matches a peer's messages to
    our receives in issue order (no tags), so a peer that is both
    neighbours (2 ranks, periodic) pairs correctly."""
    w, r = world()
    if radius == 0 or (w == 1 and not periodic):
        return
    n_owned = buf.numel() - 2 * radius
    if w == 1:  # periodic with one rank: the halos wrap onto this rank's own cells
        buf[:radius].copy_(buf[n_owned:n_owned + radius].clone())
        buf[n_owned + radius:].copy_(buf[radius:2 * radius].clone())
        return
    _transport.halo(buf, radius, periodic)
