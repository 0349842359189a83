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
  sort      (new)              exact splitting + all-to-all
  gemv      gemv.hpp:30-42                    replicate x (all_gather)
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


def world():
    return (dist.get_world_size(), dist.get_rank()) if dist.is_initialized() else (1, 0)


def _staged():
    """gloo cannot run these collectives on device tensors: stage through
    host memory (CPU tests, and the one-GPU rehearsal of the N > 1 path)."""
    return dist.get_backend() == "gloo"


def _all_gather_into(out, inp):
    if _staged() and inp.is_cuda:
        o = out.cpu()
        dist.all_gather_into_tensor(o, inp.cpu())
        out.copy_(o)
    else:
        dist.all_gather_into_tensor(out, inp)


def reduce_partials(partial, op="plus", init=None):
    """partial: 1-element tensor (the rank's segment result, ACC type).
    Returns the fold init op p_0 op p_1 ... in rank (= segment) order, on
    every rank (reduce.hpp:81-83)."""
    w, _ = world()
    if w == 1:
        return partial.clone() if init is None else OPS[op](torch.full_like(partial, init), partial)
    g = torch.empty(w, dtype=partial.dtype, device=partial.device)
    _all_gather_into(g, partial.reshape(1))
    acc = g[0:1].clone()
    for k in range(1, w):
        acc = OPS[op](acc, g[k:k + 1])
    if init is not None:
        acc = OPS[op](torch.full_like(acc, init), acc)
    return acc


def scan_carry(total, op="plus"):
    """total: 1-element tensor (the rank's segment total, ACC type).  Returns
    (carry, has_carry): the op-fold of the totals of ranks < this rank, as a
    1-element tensor on the same device (read by the scan kernel as
    carry_dev), and whether one exists (rank 0 has none)."""
    w, r = world()
    if w == 1 or r == 0:
        if w > 1:  # take part in the collective
            g = torch.empty(w, dtype=total.dtype, device=total.device)
            _all_gather_into(g, total.reshape(1))
        return None, False
    g = torch.empty(w, dtype=total.dtype, device=total.device)
    _all_gather_into(g, total.reshape(1))
    acc = g[0:1].clone()
    for k in range(1, r):
        acc = OPS[op](acc, g[k:k + 1])
    return acc, True


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
    raise TypeError(f"dist sort: unsupported key type {dt}")


def exact_splits(n_local, nbits, count_below, to_keys):
    """Exact splitting of the globally sorted order at the rank boundaries.

    n_local:     this rank's key count (the output keeps every rank's count).
    count_below: f(splitter keys ndarray[nb]) -> int64 ndarray[nb] of this
                 rank's sorted keys below each splitter (radix order).
    to_keys:     bits -> key values.
    Returns (send_counts[w], recv_counts[w]) for all_to_all_single."""
    w, r = world()
    sizes = torch.tensor([n_local], dtype=torch.int64)
    if w == 1:
        return [n_local], [n_local]
    allsz = [torch.zeros(1, dtype=torch.int64) for _ in range(w)]
    _all_gather_cpu(allsz, sizes)
    sz = [int(t.item()) for t in allsz]
    nb = w - 1
    g = np.cumsum(sz)[:nb].astype(np.int64)          # global rank of each boundary
    mask = (1 << nbits) - 1
    lo = np.zeros(nb, dtype=np.uint64)
    hi = np.full(nb, mask, dtype=np.uint64)
    for _ in range(nbits):
        c = lo + (hi - lo + 1) // 2
        below = _allreduce_sum_cpu(count_below(to_keys(c)))
        move = (below <= g) & (hi > lo)
        shrink = (below > g) & (hi > lo)
        lo = np.where(move, c, lo)
        hi = np.where(shrink, c - 1, hi)
    lt = count_below(to_keys(lo))
    le = np.where(lo == mask, n_local, count_below(to_keys(np.minimum(lo + 1, mask))))
    lt_all = _all_gather_np(lt)                      # [w, nb]
    le_all = _all_gather_np(le)
    split = np.zeros((w, nb + 1), dtype=np.int64)
    for k in range(nb):
        need = g[k] - lt_all[:, k].sum()
        for s in range(w):
            take = min(le_all[s, k] - lt_all[s, k], need)
            split[s, k] = lt_all[s, k] + take
            need -= take
    split[:, nb] = sz
    prev = np.concatenate([np.zeros((w, 1), np.int64), split[:, :nb]], axis=1)
    send = (split[r] - prev[r]).tolist()
    recv = (split[:, r] - prev[:, r]).tolist()
    return send, recv


def _all_gather_cpu(out, t):
    dev = _coll_device()
    tt = t.to(dev)
    outs = [torch.empty_like(tt) for _ in out]
    dist.all_gather(outs, tt)
    for o, x in zip(out, outs):
        o.copy_(x.cpu())


def _allreduce_sum_cpu(a):
    t = torch.from_numpy(np.ascontiguousarray(a, dtype=np.int64)).to(_coll_device())
    dist.all_reduce(t)
    return t.cpu().numpy()


def _all_gather_np(a):
    w, _ = world()
    t = torch.from_numpy(np.ascontiguousarray(a, dtype=np.int64)).to(_coll_device())
    outs = [torch.empty_like(t) for _ in range(w)]
    dist.all_gather(outs, t)
    return np.stack([o.cpu().numpy() for o in outs])


def _coll_device():
    return torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")


def dist_sort(keys, local_sort, count_below_dev, key_dtype=None, merge_runs=None):
    """Sort the distributed range whose local segment is `keys` (a 1-D
    tensor, modified in place: every rank keeps its key count).
    local_sort(t): sorts t in place on its device.
    count_below_dev(sorted_t, splitter_keys ndarray) -> int64 ndarray.
    key_dtype: numpy key type when the tensor carries other bits (uint32
    keys in an int32 tensor).
    merge_runs(t, offsets): sorts t made of the sorted runs the all-to-all
    delivered (one per source rank, offsets 0 .. n); without it the
    destination step is a second local_sort."""
    local_sort(keys)
    w, _ = world()
    if w == 1:
        return keys
    np_dt = key_dtype or {torch.int32: np.int32, torch.float32: np.float32}[keys.dtype]
    _, _, from_bits = key_bits(np_dt)
    send, recv = exact_splits(keys.numel(), 32, lambda spl: count_below_dev(keys, spl),
                              lambda bits: from_bits(bits.astype(np.uint32)))
    if _staged() and keys.is_cuda:
        src = keys.cpu()
        out = torch.empty_like(src)
        dist.all_to_all_single(out, src, output_split_sizes=recv, input_split_sizes=send)
    else:
        out = torch.empty_like(keys)
        dist.all_to_all_single(out, keys, output_split_sizes=recv, input_split_sizes=send)
    keys.copy_(out)
    if merge_runs is not None:
        merge_runs(keys, np.concatenate([[0], np.cumsum(recv)]).astype(np.int64))
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
    dev = torch.device("cpu") if (_staged() and buf.is_cuda) else buf.device
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
