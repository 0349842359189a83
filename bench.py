#!/usr/bin/env python3
"""bench.py -- Distributed Ranges shp hot path on MI355X.

Headline workload (BASELINE.json configs[1]): one STEP = shp::reduce +
shp::inclusive_scan (plus) over a distributed_vector<float> of 2^30 elements
PER GPU (weak scaling), inputs resident in HBM.  One process per GPU
(`--gpus N` starts torch.distributed.run itself when no launcher did); each
rank owns one segment and calls libdrhip.so through its C-ABI
(distributed-ranges_amd/drhip.py).  Cross-segment combines run over
libdrhip's own RCCL communicator (dr_dist.DrhipTransport: drhip_allgather /
drhip_alltoallv / drhip_halo_exchange; torch.distributed only bootstraps it
and carries the barriers):
  reduce: local drhip_reduce -> all_gather of the N fp64 partials -> fold in
          segment order by drhip_fold_partials (shp/algorithms/reduce.hpp:81-83);
  scan:   the reduce's partial is the segment total: the same all_gather
          gives the exclusive prefix of the preceding totals (fp64 for f32)
          on the device -> ONE single-pass drhip_inclusive_scan with that
          carry read by the kernel (carry_dev).  The step moves 4 + 8 B/elem
          and runs one collective at every N.

`value` = elements of the distributed vector processed per second by the
whole job (N * 2^30 / step time).  `roofline` is for the dominant kernel (the
scan): algorithmic 8 B/elem x elements per launch / mean launch time from HIP
events recorded on the drhip stream the kernel runs on.  `traffic` is the
PMC-measured HBM bytes per launch (profiles/pmc_summary.json, tools/pmc.sh).

`ops` carries the other BASELINE configs, each timed the same way
(--no-ops skips them): sort (C3: 2^28 uint32 keys per GPU, local radix sort +
exact-splitting all-to-all for N > 1), gemv (C4: 2^26-row random CSR, 10
nnz/row, rows split over the ranks, x all_gathered every call), stencil1d
(C5: 2^29 cells per GPU, 3-point, halo exchange every step).

`ops.c2_int32` is C2's integer form (bit-exact); `ops.shp_one_process` is the
reference's own execution model -- ONE process driving all N devices through
the C++ drop-in (tests/cpp/bin/shp_bench, run by rank 0).

`cpu_baseline` times the reference's CPU (mhp) execution of every BASELINE
config on the host cores, rank 0 at N = 1 only, on bounded samples
(oracle/cpu_bench: OpenMP ranks; oracle/c1_mpi_dot: C1 on 2 MPICH ranks).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "distributed-ranges_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X spec, MI355X_MICROARCH.md chip table
CPU_GROUP = None  # gloo group of all ranks (N > 1), set in main


T_START = time.time()


def log(msg):
    """progress line on stderr (a long run keeps printing)."""
    print(f"[bench {time.time() - T_START:7.1f}s] {msg}", file=sys.stderr, flush=True)


class stdout_to_stderr:
    """fd 1 -> fd 2 for a block: RCCL prints a version banner on stdout when
    a communicator is created, and the bench's stdout must hold only its one
    JSON line."""

    def __enter__(self):
        sys.stdout.flush()
        self.saved = os.dup(1)
        os.dup2(2, 1)

    def __exit__(self, *exc):
        sys.stdout.flush()
        os.dup2(self.saved, 1)
        os.close(self.saved)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--log2n", type=int, default=30, help="elements per GPU = 2^log2n")
    p.add_argument("--dtype", default="f32", choices=["f32", "i32"])
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-ops", action="store_true", help="skip the sort / gemv / stencil configs")
    p.add_argument("--only-ops", default="", help="comma list of ops to run (c2_int32,sort,gemv,stencil1d,for_each,dot,"
                   "stencil2d,dense,shp_one_process; "
                   "gemv_banded / gemv_random run one C4 kind)")
    p.add_argument("--sort-log2n", type=int, default=28)
    p.add_argument("--gemv-log2m", type=int, default=26)
    p.add_argument("--stencil-log2n", type=int, default=29)
    return p.parse_args()


PMC_CURRENT = os.path.join(ROOT, "profiles", "pmc_current.json")


def load_pmc(kernel_substr, log2n=30):
    """Per-launch HBM bytes of a kernel, and the summary they come from:
    profiles/pmc_current.json names the PMC summary measured at the code in
    the tree ({"file": ..., "commit": ...}, written with it by
    tools/pmc_summary.py --current), from rocprofv3 --pmc runs of the default
    2^30 workload, FETCH_SIZE doubled per the gfx950 correction.  (None,
    source) for any other size or kernel."""
    try:
        cur = json.load(open(PMC_CURRENT))
        path = os.path.join(ROOT, "profiles", cur["file"])
        source = {"file": "profiles/" + cur["file"], "commit": cur.get("commit")}
    except Exception:
        return None, None
    if log2n != 30:
        return None, source
    try:
        d = json.load(open(path))
        for name, v in d.get("kernels", {}).items():
            if kernel_substr in name:
                return v.get("hbm_bytes_per_launch"), source
    except Exception:
        pass
    return None, source


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(dtype):
    """The reference's CPU execution of every BASELINE config, timed on this
    box's host cores (rank 0, N = 1 only): oracle/cpu_bench (C2-C5, OpenMP
    threads playing the mhp ranks) and oracle/c1_mpi_dot (C1 on 2 MPICH
    ranks).  Median of 7 runs each after a warm-up; bounded samples (2^27
    elements, 2^24 keys, 2^22 CSR rows, 2^27 stencil cells).  The top-level
    value is C2, the headline config."""
    import subprocess
    odir = os.path.join(ROOT, "oracle")
    # this GPU's share of the host: the GPU box allots 16 CPUs to a one-GPU
    # job (it exports OMP_NUM_THREADS=16; nproc shows the whole machine)
    cores = int(os.environ.get("OMP_NUM_THREADS") or min(16, os.cpu_count() or 1))
    out = {}
    r = subprocess.run([os.path.join(odir, "cpu_bench"), str(cores), "7"], capture_output=True, text=True,
                       timeout=240)
    if r.returncode != 0:
        raise RuntimeError(f"cpu_bench failed: {r.stderr[-400:]}")
    for line in r.stdout.splitlines():
        if line.startswith("{"):
            d = json.loads(line)
            out[d.pop("config")] = d
    mpiexec = "/opt/conda/bin/mpiexec"
    c1 = os.path.join(odir, "c1_mpi_dot")
    if os.path.exists(mpiexec) and os.path.exists(c1):
        try:
            r = subprocess.run([mpiexec, "-n", "2", c1, "24", "7"], capture_output=True, text=True, timeout=60)
            for line in r.stdout.splitlines():
                if line.startswith("{"):
                    d = json.loads(line)
                    out[d.pop("config")] = d
            if "C1" not in out:
                out["C1"] = {"error": (r.stderr or r.stdout)[-300:]}
        except subprocess.TimeoutExpired:
            out["C1"] = {"error": "mpiexec timed out"}
    c2 = out["C2"]
    return {"value": c2["value"], "unit": c2["unit"], "cores": cores, "kind": "port",
            "cpu_model": cpu_model(), "host_cpus": os.cpu_count(),
            "sample": f"C2: {c2['workload']} on {cores} OpenMP ranks, median of {c2['runs']} runs "
                      f"(oracle/cpu_bench); every config below, C1 on 2 MPICH ranks",
            "cores_note": "one thread per CPU of the GPU box's allotment for this GPU (OMP_NUM_THREADS)",
            "configs": out}


def max_rel_err(torch, got, ref, chunk=1 << 27):
    """max |got - ref| / |ref| on the device, chunked (fp64 refs of 2^30)."""
    e = 0.0
    for i in range(0, ref.numel(), chunk):
        r = ref[i:i + chunk]
        d = (got[i:i + chunk].double() - r).abs() / r.abs().clamp_min(1e-30)
        e = max(e, float(d.max().item()))
    return e


def check_reduce_scan(torch, x, out, red_part, carry, world, rank, dtype):
    """Headline checks: this rank's reduce partial and every element of its
    scanned segment (carry included at N > 1)."""
    if dtype == "f32":
        ref_sum = float(x.double().sum().item())
        r_err = abs(float(red_part.item()) - ref_sum) / abs(ref_sum)
        ref = torch.cumsum(x.double(), 0)
        if carry is not None:
            ref += float(carry.item())
        s_err = max_rel_err(torch, out, ref)
        del ref
        return {"reduce_rel_err": r_err, "scan_max_rel_err": s_err, "tolerance": 1e-5,
                "ok": bool(r_err <= 1e-5 and s_err <= 1e-5), "scope": "every element, rank %d" % rank}
    ref = torch.cumsum(x, 0, dtype=torch.int64)
    if carry is not None:
        ref += int(carry.item())
    bad = int((ref.to(torch.int32) != out).sum().item())
    r_ok = (int(x.long().sum().item()) - int(red_part.item())) % (1 << 32) == 0
    del ref
    return {"reduce_exact": r_ok, "scan_mismatches": bad, "ok": bool(r_ok and bad == 0),
            "scope": "every element, rank %d (wrapping int32)" % rank}


def all_ranks(torch, dist, world, check):
    """Fold every rank's check into rank 0's line at N > 1: ok only if ok on
    every rank (rank 0's segment has no carry; ranks > 0 check theirs)."""
    if world > 1 and isinstance(check, dict) and "ok" in check:
        t = torch.tensor([1.0 if check["ok"] else 0.0], dtype=torch.float64,
                         device="cuda" if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        check["ok_all_ranks"] = bool(t.item() == 1.0)
        check["scope"] = check.get("scope", "") + "; ok folded over all %d ranks" % world
        check["ok"] = check["ok"] and check["ok_all_ranks"]
    return check


def check_sort(torch, dist, src, keys, world):
    """uint32 keys carried in int32 tensors.  N = 1: equal to torch.sort of
    the input in unsigned order (sorted AND a permutation).  N > 1: locally
    sorted, rank boundaries ordered, and the global multiset of keys equal
    (sum and xor of a 64-bit mix of every key, all-reduced)."""
    flip = torch.tensor(-(1 << 31), dtype=torch.int32, device=keys.device)
    if world == 1:
        ref = (torch.sort(src ^ flip).values) ^ flip
        bad = int((ref != keys).sum().item())
        return {"mismatches": bad, "ok": bad == 0, "ref": "torch.sort (unsigned order), every key"}
    u = (keys ^ flip)  # signed order == unsigned order of the keys
    local_sorted = bool((u[1:] >= u[:-1]).all().item())

    def mix(t):
        z = t.long() & 0xFFFFFFFF
        z = (z * (0x9E3779B97F4A7C15 - (1 << 64))) ^ (z >> 29)
        return (z * (0xBF58476D1CE4E5B9 - (1 << 64))) ^ (z >> 31)
    h = torch.stack([mix(src).sum(), mix(keys).sum()])
    dist.all_reduce(h)
    ends = torch.stack([u[0], u[-1]]).to(torch.int64)
    allends = [torch.empty_like(ends) for _ in range(world)]
    dist.all_gather(allends, ends)
    e = torch.stack(allends).cpu().tolist()
    bounds_ok = all(e[i][1] <= e[i + 1][0] for i in range(world - 1))
    # global ranks of this rank's first and last output keys: in a correct
    # sort the key at global position g satisfies #(keys < v) <= g <
    # #(keys <= v), counted over EVERY rank's input.  With local order and
    # the multiset equality this pins the output to the exact sorted
    # sequence (any correct sort of the same keys gives the same bits).
    # (every rank counts its input against every rank's first / last key)
    su = src ^ flip
    cnt = torch.stack([torch.stack([(su < e[j][0]).sum(), (su <= e[j][0]).sum(), (su < e[j][1]).sum(),
                                    (su <= e[j][1]).sum()]) for j in range(world)])
    dist.all_reduce(cnt)
    sizes = [torch.zeros(1, dtype=torch.int64, device=keys.device) for _ in range(world)]
    dist.all_gather(sizes, torch.tensor([keys.numel()], dtype=torch.int64, device=keys.device))
    me = dist.get_rank()
    g0 = sum(int(t.item()) for t in sizes[:me])
    c = [int(v) for v in cnt[me].cpu().tolist()]
    ranks_ok = c[0] <= g0 < c[1] and c[2] <= g0 + keys.numel() - 1 < c[3]
    ok = local_sorted and bounds_ok and ranks_ok and int(h[0].item()) == int(h[1].item())
    return {"locally_sorted": local_sorted, "rank_bounds_ordered": bounds_ok, "global_ranks_exact": ranks_ok,
            "multiset_hash_equal": int(h[0].item()) == int(h[1].item()), "ok": bool(ok),
            "ref": "local order + multiset hash + the global rank of every rank's first and last key"}


def check_gemv(torch, rowptr, colind, vals, xf, y, nnz):
    """y (one call from 0) vs fp64 rows built by torch from the same CSR."""
    rows = rowptr.numel() - 1
    row_of = torch.repeat_interleave(torch.arange(rows, device=y.device), (rowptr[1:] - rowptr[:-1]).long())
    ref = torch.zeros(rows, dtype=torch.float64, device=y.device)
    ref.index_add_(0, row_of, vals[:nnz].double() * xf[colind[:nnz].long()].double())
    err = max_rel_err(torch, y, ref)
    del row_of, ref
    return {"max_rel_err": err, "tolerance": 1e-5, "ok": err <= 1e-5, "ref": "torch fp64 CSR rows, every row"}


class Timer:
    """HIP events recorded on the drhip stream around each timed op."""

    def __init__(self, torch, stream):
        self.torch, self.stream, self.ev = torch, stream, {}

    def __call__(self, name, fn, record=True):
        if not record:
            return fn()
        e0 = self.torch.cuda.Event(enable_timing=True)
        e1 = self.torch.cuda.Event(enable_timing=True)
        e0.record(self.stream)
        r = fn()
        e1.record(self.stream)
        self.ev.setdefault(name, []).append((e0, e1))
        return r

    def ms(self, name):
        v = self.ev.get(name)
        return sum(a.elapsed_time(b) for a, b in v) / len(v) if v else None


def agree(torch, dist, world, ok):
    """Every rank's `ok` folded with MIN over the host-side (gloo) group, so
    all ranks take the same branch into the same next collective."""
    if world == 1:
        return bool(ok)
    t = torch.tensor([1 if ok else 0], dtype=torch.int32)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=CPU_GROUP)
    return bool(t.item() == 1)


def graph_phase(torch, dist, world, rank, capture, launch, destroy, timed):
    """Capture one step as a graph, warm it up, time its replays: returns
    (ms per replay, None) or (None, error text).  Rank-symmetric on failure:
    a rank whose capture or warm-up replay failed must not leave the others
    inside a captured collective or a barrier, so every rank folds its
    success into one host-side MIN (`agree`) before each phase and all take
    the same branch.  DRHIP_BENCH_FAIL_CAPTURE_RANK=r makes rank r's capture
    fail (tests/test_dist_gloo.py, tools/bench_2rank_1gpu.sh)."""
    ge, err = None, None
    try:
        ge = capture(os.environ.get("DRHIP_BENCH_FAIL_CAPTURE_RANK") == str(rank))
    except Exception as e:  # noqa: BLE001 -- reported
        err = f"capture: {type(e).__name__}: {e}"[:300]
    ms = None
    try:
        ok = agree(torch, dist, world, err is None)
        if ok:
            try:
                for _ in range(2):
                    launch(ge)
                torch.cuda.synchronize()
            except Exception as e:  # noqa: BLE001 -- reported
                err = f"replay: {type(e).__name__}: {e}"[:300]
            ok = agree(torch, dist, world, err is None)
        if ok:
            ms = timed(lambda: launch(ge))
    finally:
        if ge:
            torch.cuda.synchronize()
            destroy(ge)
    return ms, (None if ms is not None else err or "graph capture or replay failed on another rank")


def timed_region(torch, dist, world, fn, steps):
    """barrier + sync on both sides, max over ranks (ms per call)."""
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device="cuda" if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    return dt / steps * 1e3


def self_launch(args):
    """`bench.py --gpus N` (N > 1) started without a launcher: start N ranks
    with torch.distributed.run as a CHILD process (nothing here has touched
    the GPU; no exec) and return its exit code.  Rank 0 prints the line."""
    import socket
    import subprocess
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.run(cmd).returncode


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return self_launch(args)
    import numpy as np
    import torch
    import torch.distributed as dist
    import drhip
    import dr_dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("DRHIP_FORCE_LOCAL0"):  # tools/bench_2rank_1gpu.sh rehearsal only
        local = 0
    torch.cuda.set_device(local)
    backend = None
    transport_note = ""
    if world > 1:
        backend = os.environ.get("DRHIP_BENCH_BACKEND", "nccl")  # gloo: one-GPU rehearsal only
        if backend == "nccl":
            with stdout_to_stderr():  # eager communicator: RCCL's banner
                dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
        # host-side group for waits that must not put a spinning collective
        # kernel on the GPUs (rank 0's one-process shp_bench uses them all)
        global CPU_GROUP
        CPU_GROUP = dist.new_group(backend="gloo")

    log(f"rank {rank}/{world} on device {local}")
    # this rank's segment: one per GPU; at N > 1 a second segment on the same
    # device gives the stencils a second stream, so the interior cells are
    # computed while segment 0 exchanges the halos
    drhip.init([local, local] if world > 1 else [local])
    stream = torch.cuda.ExternalStream(drhip.stream(0))
    if backend == "nccl":
        # every cross-segment exchange below goes through libdrhip's own RCCL
        # communicator (drhip_allgather / drhip_alltoallv /
        # drhip_halo_exchange on the segment stream); torch.distributed only
        # carries the unique id, the barriers and the max-over-ranks timing
        # If any rank's communicator cannot be built, every rank falls back
        # to torch.distributed (also RCCL) and the line says so in
        # config.combine: a transport failure must not cost the measurement.
        tr, why = None, ""
        try:
            with stdout_to_stderr():
                tr = dr_dist.DrhipTransport.bootstrap(0, stream=stream)
        except Exception as e:  # noqa: BLE001 -- reported in the JSON line
            why = f"{type(e).__name__}: {e}"[:200]
        ok = torch.tensor([1 if tr is not None else 0], dtype=torch.int32, device="cuda")
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        if int(ok.item()) == 1:
            dr_dist.use(tr)
        else:
            transport_note = f" (drhip communicator unavailable on some rank{': ' + why if why else ''})"
    T = Timer(torch, stream)
    n = 1 << args.log2n
    dt_np = np.dtype({"f32": "float32", "i32": "int32"}[args.dtype])
    tdt = {"f32": torch.float32, "i32": torch.int32}[args.dtype]
    acc_t = torch.float64 if args.dtype == "f32" else torch.int32

    with torch.cuda.stream(stream):
        g = torch.Generator(device="cuda").manual_seed(1 + rank)
        if args.dtype == "f32":
            x = torch.rand(n, generator=g, device="cuda", dtype=tdt)
        else:
            x = torch.randint(0, 1 << 16, (n,), generator=g, device="cuda", dtype=tdt)
        out = torch.empty_like(x)
        red_part = torch.zeros(1, dtype=acc_t, device="cuda")
        gathered = torch.zeros(world, dtype=acc_t, device="cuda")
        result = torch.zeros(1, dtype=acc_t, device="cuda")
    torch.cuda.synchronize()
    held = {}

    def step(record):
        with torch.cuda.stream(stream):
            # ---- shp::reduce: drhip_reduce_tiles reads the range in the
            # scan's tiles and leaves each tile's exclusive prefix behind
            T("reduce", lambda: drhip.reduce_tiles_async(0, dt_np, "plus", x.data_ptr(), n, red_part.data_ptr()),
              record)
            # ---- shp::inclusive_scan over the same range: no look-back
            # (the tile prefixes come from the reduce).  N > 1: the
            # reduce's segment partial IS this segment's scan total, so ONE
            # all_gather of the N partials gives both the reduce result and
            # the scan carry, folded by the scan kernel itself (its carry:
            # ranks < rank; `result`: all N); 4 + 8 B/elem at every N
            if world > 1:
                dr_dist.gather_partials(red_part, gathered)
                T("scan", lambda: drhip.scan_tiles_async(0, dt_np, "plus", x.data_ptr(), out.data_ptr(), n,
                                                         partials=gathered.data_ptr(), w=world, rank=rank,
                                                         result=result.data_ptr()), record)
            else:
                T("scan", lambda: drhip.scan_tiles_async(0, dt_np, "plus", x.data_ptr(), out.data_ptr(), n), record)

    for _ in range(args.warmup):
        step(False)
    dt = timed_region(torch, dist, world, lambda: step(True), args.steps) * args.steps * 1e-3
    drhip.sync(0)  # surfaces an in-kernel timeout, if any

    log(f"headline: {dt / args.steps * 1e3:.4f} ms/step")
    ms_red, ms_scan = T.ms("reduce"), T.ms("scan")
    isz = dt_np.itemsize

    # the standalone single-pass scan (drhip_inclusive_scan: decoupled
    # look-back, what a scan without a preceding reduce of its range runs),
    # timed on the same input for comparison
    with torch.cuda.stream(stream):
        for _ in range(2):
            drhip.scan_async(0, dt_np, "plus", x.data_ptr(), out.data_ptr(), n)
        for _ in range(max(3, min(args.steps, 10))):
            T("scan_single_pass", lambda: drhip.scan_async(0, dt_np, "plus", x.data_ptr(), out.data_ptr(), n))
    torch.cuda.synchronize()
    ms_sp = T.ms("scan_single_pass")
    # checks (outside the timed region, independent of the oracle): the
    # reduce vs torch's fp64 sum, EVERY scanned element vs torch's fp64
    # cumsum (f32: rel <= 1e-5) or its wrapped int64 cumsum (i32: exact),
    # for the step's output (rerun: the timing loop above overwrote `out`)
    with torch.cuda.stream(stream):
        step(False)
        drhip.reduce_async(0, dt_np, "plus", x.data_ptr(), n, red_part.data_ptr())
    torch.cuda.synchronize()
    carry_chk = None
    if world > 1 and rank > 0:  # the carry the scan folded: the gathered partials of ranks < rank
        carry_chk = gathered[:rank].double().sum().to(acc_t).reshape(1) if args.dtype == "f32" else \
            gathered[:rank].long().sum().reshape(1)
    check = all_ranks(torch, dist, world, check_reduce_scan(torch, x, out, red_part, carry_chk, world, rank,
                                                            args.dtype))
    if world > 1:
        tot = float(gathered.double().sum().item()) if args.dtype == "f32" else int(gathered.long().sum().item())
        check["reduce_result_ok"] = bool(abs(float(result.item()) - tot) <= 1e-9 * max(1.0, abs(tot))) \
            if args.dtype == "f32" else (int(result.item()) - tot) % (1 << 32) == 0
        check["ok"] = check["ok"] and check["reduce_result_ok"]
    del out, x
    torch.cuda.empty_cache()

    scan_bytes = 2 * isz * n
    achieved = scan_bytes / (ms_scan * 1e-3) / 1e9
    # the instantiations the 2^30 step launches (big tiles: 32 vectors per thread)
    ctype = "float" if args.dtype == "f32" else "int"
    scan_kname = f"scan_wave_given_kernel<0, {ctype}, true, 32, 256>"
    ops = {
        "reduce": {"ms": ms_red, "elements_per_s": n / (ms_red * 1e-3),
                   "GBps": isz * n / (ms_red * 1e-3) / 1e9,
                   "frac": isz * n / (ms_red * 1e-3) / 1e9 / HBM_PEAK_GBS,
                   "traffic": load_pmc(f"reduce_tiles_kernel<0, {ctype}, 32>", args.log2n)[0],
                   "kernel": "reduce_tiles_kernel (drhip_reduce_tiles)"},
        "inclusive_scan": {"ms": ms_scan, "elements_per_s": n / (ms_scan * 1e-3), "GBps": achieved,
                           "frac": achieved / HBM_PEAK_GBS,
                           "kernel": "scan_wave_given_kernel (tile-part prefixes from the step's reduce: no look-back, no LDS, no barrier)"},
        "inclusive_scan_single_pass": {"ms": ms_sp, "frac": scan_bytes / (ms_sp * 1e-3) / 1e9 / HBM_PEAK_GBS,
                                       "kernel": "scan_kernel (decoupled look-back; drhip_inclusive_scan alone)"},
    }
    if not args.no_ops:
        ops.update(extra_ops(args, torch, dist, np, drhip, dr_dist, stream, world, rank))

    res = {
        "metric": "elements/s & % HBM roofline: reduce/scan/sort/SpMV at 1/2/4/8 MI355X",
        "value": world * n * args.steps / dt,
        "unit": "elements/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": dt / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": args.dtype,
        "data": "synthetic (torch.rand U[0,1) on device, seed 1+rank)" if args.dtype == "f32"
                else "synthetic (U[0,2^16) int32 on device, seed 1+rank)",
        "config": {"workload": f"shp reduce + inclusive_scan (plus), distributed_vector<"
                               f"{'float' if args.dtype == 'f32' else 'int32'}> 2^{args.log2n} elements per GPU, "
                               f"one segment per GPU",
                   "elements_per_gpu": n, "global_elements": world * n,
                   "parallelism": f"segments{world}",
                   "combine": (f"all_gather of the N partials over {dr_dist.transport().name}{transport_note},"
                               f" folded by the scan kernel (drhip_inclusive_scan_tiles with the gathered partials)"
                               if world > 1 else "none")},
        "roofline": {"bound": "hbm", "kernel": "drhip::scan_wave_given_kernel (the step's scan: each wave part's prefix "
                                               "from the step's reduce, no look-back, no LDS, no barrier)",
                     "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS,
                     "traffic": load_pmc(scan_kname, args.log2n)[0],
                     "traffic_source": dict(load_pmc(scan_kname, args.log2n)[1] or {}, kernel=scan_kname),
                     "algorithmic_bytes_per_launch": scan_bytes,
                     "launch_ms": ms_scan},
        "ops": ops,
        "check": check,
    }
    log("ops done")
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        res["cpu_baseline"] = cpu_baseline(args.dtype)
    elif rank == 0:
        res["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(res), flush=True)
    drhip.finalize()
    if world > 1:
        dist.destroy_process_group()
    return 0


def c2_strong(args, torch, dist, np, drhip, dr_dist, stream, world, rank, steps):
    """C2 under STRONG scaling -- the north star's 7x target is quoted on ONE
    2^30-element fp32 distributed_vector: 2^log2n elements in total, split
    ceil(n/N) per rank (shp/distributed_vector.hpp:142), one step = reduce +
    inclusive_scan with the combine (all_gather of the N partials + fold in
    segment order) inside the timed region.

    Two launch modes of the same step: `eager` (one C-ABI call per kernel,
    as the headline) and `graph` (the step captured once with
    drhip_graph_begin/end -- reduce kernel, RCCL all_gather, fold kernel,
    scan memset + kernel -- and replayed with one drhip_graph_launch per
    step: every kernel still runs every step, only the host launch gaps go).

    At N = 1 it also times the per-rank critical path of the N = 8 job on
    this one GPU: 2^(log2n-3) elements with a one-rank libdrhip RCCL
    communicator doing the all_gather + drhip_fold_partials in the step
    exactly as every rank does at N = 8 (`per_rank_of_8`), and from it the
    predicted 8-GPU strong speed-up (RCCL's 8-rank all_gather latency
    excepted, which one GPU cannot measure).  Timed like the headline:
    barrier + sync around K steps, max over ranks; kernel times from HIP
    events on the segment stream (eager mode)."""
    T = Timer(torch, stream)
    n_tot = 1 << args.log2n
    per = (n_tot + world - 1) // world
    n = max(0, min(n_tot, (rank + 1) * per) - rank * per)
    gsteps = max(steps, 20)

    def run(n_local, w, r, gather):
        """gather(part, g): all_gather of the 1-element partial into g[w]
        (None: no combine); the scan kernel then folds the gathered partials
        itself (drhip_inclusive_scan_tiles with the gathered partials: carry =
        fold of ranks < r, result = fold of all).  Returns eager + graph timings and the check."""
        with torch.cuda.stream(stream):
            g = torch.Generator(device="cuda").manual_seed(31 + rank)
            x = torch.rand(n_local, generator=g, device="cuda")
            out = torch.empty_like(x)
            part = torch.zeros(1, dtype=torch.float64, device="cuda")
            gat = torch.zeros(w, dtype=torch.float64, device="cuda")
            res = torch.zeros(1, dtype=torch.float64, device="cuda")
            carry = torch.zeros(1, dtype=torch.float64, device="cuda")
        has = gather is not None and r > 0

        def body(record):
            T("reduce", lambda: drhip.reduce_tiles_async(0, np.float32, "plus", x.data_ptr(), n_local,
                                                         part.data_ptr()), record)
            if gather is not None:
                gather(part, gat)
                T("scan", lambda: drhip.scan_tiles_async(0, np.float32, "plus", x.data_ptr(), out.data_ptr(),
                                                         n_local, partials=gat.data_ptr(), w=w, rank=r,
                                                         result=res.data_ptr()), record)
            else:
                T("scan", lambda: drhip.scan_tiles_async(0, np.float32, "plus", x.data_ptr(), out.data_ptr(),
                                                         n_local), record)

        def step():
            with torch.cuda.stream(stream):
                body(True)

        for _ in range(2):
            step()
        T.ev.clear()
        ms = timed_region(torch, dist, world, step, steps)
        torch.cuda.synchronize()
        out_r = {"ms": ms, "reduce_kernel_ms": T.ms("reduce"), "scan_kernel_ms": T.ms("scan")}
        T.ev.clear()
        # graph mode: capture one step, replay it (rank-symmetric on failure)
        def capture(inject):
            with torch.cuda.stream(stream):
                drhip.graph_begin(0)
                ge = None
                try:
                    if inject:
                        raise RuntimeError("injected capture failure (DRHIP_BENCH_FAIL_CAPTURE_RANK)")
                    body(False)
                finally:
                    ge = drhip.graph_end(0)
            return ge

        gms, gerr = graph_phase(torch, dist, world, rank, capture, lambda ge: drhip.graph_launch(0, ge),
                                drhip.graph_destroy, lambda fn: timed_region(torch, dist, world, fn, gsteps))
        if gms is not None:
            out_r["graph_ms"] = gms
        else:
            out_r["graph_error"] = gerr
            step()  # the eager step again, so the check below covers this rank's outputs
        torch.cuda.synchronize()
        # the check covers the last (graph or eager) step's outputs
        if has:  # this rank's carry, for the check: the fold of the gathered partials before it
            carry.fill_(float(gat[:r].double().sum().item()))
        out_r["check"] = check_reduce_scan(torch, x, out, part, carry if has else None, world, rank, "f32")
        all_ranks(torch, dist, w, out_r["check"])
        if gather is not None:
            ref = float(x.double().sum().item())  # this rank's partial; the fold of all is checked at w = 1
            out_r["check"]["fold_ok"] = bool(w > 1 or abs(float(res.item()) - ref) <= 1e-5 * abs(ref))
            out_r["check"]["ok"] = out_r["check"]["ok"] and out_r["check"]["fold_ok"]
        del x, out, part, gat, res, carry
        torch.cuda.empty_cache()
        return out_r

    tr = dr_dist.transport()
    if world > 1 and not isinstance(tr, dr_dist.DrhipTransport):
        gather = None  # gloo / torch fallback: no capturable collective
        r = run(n, world, rank, None)
        r["note"] = f"combine skipped: {tr.name} cannot be captured"
    else:
        r = run(n, world, rank, (lambda part, g: tr.all_gather_into(g, part)) if world > 1 else None)
    if world > 1:
        # the same step with the collective-free combine: flag slots mapped
        # across the rank processes (dr_dist.FlagSlots, drhip_xchg_allgather)
        fs, why = None, ""
        try:
            fs = dr_dist.FlagSlots.bootstrap(0, group=CPU_GROUP)
        except Exception as e:  # noqa: BLE001 -- reported
            why = f"{type(e).__name__}: {e}"[:300]
        if agree(torch, dist, world, fs is not None):
            rf = run(n, world, rank, lambda part, g: fs.all_gather_into(g, part))
            try:
                drhip.sync(0)  # a wait past the spin bound surfaces here
            except Exception as e:  # noqa: BLE001 -- reported
                rf["error"] = f"{type(e).__name__}: {e}"[:300]
                rf["check"]["ok"] = False
            all_ranks(torch, dist, world, rf["check"])
            rf["combine"] = fs.name
            dist.barrier(group=CPU_GROUP)
            fs.close()
            r["flags"] = rf
        else:
            r["flags"] = {"error": why or "flag slots unavailable on another rank"}
    best = min(r["ms"], r.get("graph_ms", r["ms"]))
    fl = r.get("flags", {})
    if isinstance(fl, dict) and fl.get("check", {}).get("ok"):
        best = min(best, fl["ms"], fl.get("graph_ms", fl["ms"]))
    r.update({"config": f"shp reduce + inclusive_scan (plus), distributed_vector<float> 2^{args.log2n} elements IN TOTAL "
                        f"over {world} GPU(s) (ceil(n/N) = {per} per GPU), combine inside the timed step",
              "elements_per_s": n_tot / (best * 1e-3), "eager_elements_per_s": n_tot / (r["ms"] * 1e-3),
              "scaling": "strong",
              "combine": (f"all_gather of the N partials over {tr.name}, folded by the scan kernel "
                          f"(drhip_inclusive_scan_tiles with the gathered partials)" if world > 1 else "none")})
    if world == 1 and args.log2n >= 3:
        # one-rank libdrhip RCCL communicator: the all_gather + fold of every
        # rank's step at N = 8, on this GPU (the folded value is read by the
        # scan as its carry, as ranks > 0 do)
        nr = n_tot >> 3
        try:
            with stdout_to_stderr():
                drhip.comm_init_rank(0, 1, 0, drhip.comm_unique_id())
        except Exception as e:  # noqa: BLE001 -- reported
            r["per_rank_of_8"] = {"error": f"{type(e).__name__}: {e}"[:200]}
            return r
        try:
            q = run(nr, 1, 0, lambda part, g: drhip.allgather(0, part.data_ptr(), g.data_ptr(), 8))
        finally:
            drhip.comm_destroy(0)
        nocomb = run(nr, 1, 0, None)
        qb = min(q["ms"], q.get("graph_ms", q["ms"]))
        nb = min(nocomb["ms"], nocomb.get("graph_ms", nocomb["ms"]))
        # the flag-slot combine on one rank (its own slot only): the exchange
        # kernel's cost in the step; cross-GPU latency needs N > 1
        try:
            slots = drhip.xchg_alloc(0, 1)
            try:
                qf = run(nr, 1, 0, lambda part, g: drhip.xchg_allgather(0, slots, [slots], 0, part.data_ptr(),
                                                                        g.data_ptr()))
                drhip.sync(0)
            finally:
                drhip.xchg_free(0, slots)
            qfb = min(qf["ms"], qf.get("graph_ms", qf["ms"]))
            qf.update({"combine_ms": qfb - nb, "combine": "one-rank flag-slot exchange (drhip_xchg_allgather)"})
            r["per_rank_of_8_flags"] = qf
        except Exception as e:  # noqa: BLE001 -- reported
            r["per_rank_of_8_flags"] = {"error": f"{type(e).__name__}: {e}"[:300]}
        q.update({"elements": nr, "ms_without_combine": nocomb["ms"], "graph_ms_without_combine":
                  nocomb.get("graph_ms"), "combine_ms": qb - nb,
                  "combine": "one-rank libdrhip RCCL all_gather (drhip_allgather); the scan kernel folds the "
                             "gathered partials (drhip_inclusive_scan_tiles)"})
        r["per_rank_of_8"] = q
        # upper bounds: a one-rank combine has no cross-GPU latency; the range
        # adds the 20-40 us an 8-rank all_gather over xGMI takes (DESIGN 6.1,
        # an assumption: 8 GPUs are not measurable here)
        r["predicted_speedup_8_upper_bound"] = best / qb
        r["predicted_speedup_8_range"] = [best / (qb + 0.040), best / (qb + 0.020)]
        qf = r.get("per_rank_of_8_flags", {})
        if qf.get("check", {}).get("ok"):
            r["predicted_speedup_8_flags_upper_bound"] = best / min(qf["ms"], qf.get("graph_ms", qf["ms"]))
        r["predicted_note"] = ("upper bound = best ms(2^%d on 1 GPU) / best ms(per-rank step of N = 8 with a one-rank "
                               "combine), which has no cross-GPU latency; range = the same with 20-40 us of 8-rank "
                               "all_gather latency added (assumed, not measured)" % args.log2n)
    return r


def overlap_step(torch, stream, stream1, interior, rest):
    """One stencil step with the halo exchange hidden under the interior:
    segment 1's stream (same GPU) waits for everything queued so far on
    segment 0's, runs `interior`; segment 0 runs `rest` (exchange + edge
    cells) meanwhile; segment 0 then waits for segment 1, so the next step
    (and the timed region's end) sees both."""
    e0 = torch.cuda.Event()
    e0.record(stream)
    stream1.wait_event(e0)
    with torch.cuda.stream(stream1):
        interior()
    with torch.cuda.stream(stream):
        rest()
    e1 = torch.cuda.Event()
    e1.record(stream1)
    stream.wait_event(e1)


def extra_ops(args, torch, dist, np, drhip, dr_dist, stream, world, rank):
    ops = {}
    T = Timer(torch, stream)
    stream1 = torch.cuda.ExternalStream(drhip.stream(1)) if world > 1 else None
    T1 = Timer(torch, stream1) if world > 1 else T
    steps = max(3, min(args.steps, 10))

    def want(k):
        w = not args.only_ops or k in args.only_ops.split(",")
        if w:
            log(f"op {k}")
        return w
    nc = 1 << args.stencil_log2n  # cells per GPU of the stencil / for_each configs

    # ----------------------------------- C2 int32 (the bit-exact C2 variant)
    if want("c2_int32") and args.dtype == "f32":
        n = 1 << args.log2n
        with torch.cuda.stream(stream):
            gi = torch.Generator(device="cuda").manual_seed(21 + rank)
            xi = torch.randint(0, 1 << 16, (n,), generator=gi, device="cuda", dtype=torch.int32)
            oi = torch.empty_like(xi)
            pi = torch.zeros(1, dtype=torch.int32, device="cuda")
        held = {}

        def c2i_step():
            with torch.cuda.stream(stream):
                # the headline's step in int32: tile-prefix reduce, then the
                # scan with the carry fold of the all_gathered partials
                T("reduce_i32", lambda: drhip.reduce_tiles_async(0, np.int32, "plus", xi.data_ptr(), n,
                                                                 pi.data_ptr()))
                cp = None
                if world > 1:
                    _, c, has = dr_dist.reduce_and_carry(pi, "plus")
                    if has:
                        held["carry"] = c
                        cp = c.data_ptr()
                T("scan_i32", lambda: drhip.scan_tiles_async(0, np.int32, "plus", xi.data_ptr(), oi.data_ptr(), n,
                                                             carry_dev=cp))

        c2i_step()
        T.ev.clear()
        ms = timed_region(torch, dist, world, c2i_step, steps)
        ms_r, ms_s = T.ms("reduce_i32"), T.ms("scan_i32")
        torch.cuda.synchronize()
        check = all_ranks(torch, dist, world, check_reduce_scan(torch, xi, oi, pi, held.get("carry"), world, rank,
                                                                "i32"))
        ops["c2_int32"] = {"config": f"shp reduce + inclusive_scan (plus), distributed_vector<int32> 2^{args.log2n} "
                                     f"elements per GPU, U[0,2^16), wrapping int32 (C2's integer form)",
                           "ms": ms, "elements_per_s": world * n / (ms * 1e-3),
                           "reduce_ms": ms_r, "reduce_frac": 4.0 * n / (ms_r * 1e-3) / 1e9 / HBM_PEAK_GBS,
                           "scan_ms": ms_s, "scan_frac": 8.0 * n / (ms_s * 1e-3) / 1e9 / HBM_PEAK_GBS,
                           "check": check, "scaling": "weak"}
        del xi, oi, pi, held
        torch.cuda.empty_cache()

    # ------------------------------- C2 strong scaling (2^log2n in TOTAL)
    if want("c2_strong") and args.dtype == "f32":
        ops["c2_strong"] = c2_strong(args, torch, dist, np, drhip, dr_dist, stream, world, rank, steps)

    # ------------------------------------------------------------ C3 sort
    if want("sort"):
        ns = 1 << args.sort_log2n
        with torch.cuda.stream(stream):
            gen = torch.Generator(device="cuda").manual_seed(77 + rank)
            src = torch.randint(-(1 << 31), 1 << 31, (ns,), generator=gen, device="cuda", dtype=torch.int32)
            keys = torch.empty_like(src)
            wsb = max(drhip.sort_workspace(0, np.uint32, ns), drhip.merge_workspace(0, np.uint32, ns, world))
            ws = torch.empty(wsb, dtype=torch.uint8, device="cuda")

        # uint32 keys are carried in int32 tensors (torch has no uint32 ops);
        # every kernel is told the dtype is uint32, and dr_dist sorts by the
        # unsigned (radix) order through key_bits(np.uint32).
        def local_sort(t):
            T("sort_local", lambda: drhip.sort_async(0, np.uint32, t.data_ptr(), t.numel(), ws.data_ptr(), wsb))

        def merge_into(a, b, offs):  # the all_to_all's landing buffer -> the segment, no copies
            T("sort_merge", lambda: drhip.merge_runs_to(0, np.uint32, a.data_ptr(), b.data_ptr(), b.numel(), offs,
                                                        ws.data_ptr(), wsb))

        land = torch.empty_like(keys) if world > 1 else None

        def sort_step():
            with torch.cuda.stream(stream):
                T("sort_input_copy", lambda: keys.copy_(src))  # fresh unsorted input, reported separately
                dr_dist.dist_sort(keys, local_sort, key_dtype=np.uint32, merge_into=merge_into, landing=land)

        sort_step()
        T.ev.clear()
        ms = timed_region(torch, dist, world, sort_step, steps)
        ms_local = T.ms("sort_local")
        ms_copy = T.ms("sort_input_copy")
        check = check_sort(torch, dist, src, keys, world)
        # sort.hip's shipped policy: onesweep (one tile-histogram read for the
        # pass-0 bases + 4 rank/look-back/scatter passes = 4 + 4 x 8 = 36 B/key) from 256 MiB of
        # keys, the classic per-pass histogram path (4 x 12 = 48 B/key) below
        onesweep = ns * 4 >= (1 << 28)
        bpk = 36.0 if onesweep else 48.0
        ops["sort"] = {"config": f"2^{args.sort_log2n} uint32 keys per GPU (C3 weak), LSD radix 4 x 8-bit passes"
                                 + (" (onesweep: pass-0 digit bases from a tile histogram, decoupled look-back digit offsets in passes 1-3, 16 K-key tiles claimed in groups of 64 per XCD)" if onesweep else "")
                                 + (", exact splitting from 2 small allgathers (regular samples, boundary slices) + all_to_all over RCCL into a landing buffer + merge-path merge of the received runs straight into the segment" if world > 1 else ""),
                       "ms": ms, "keys_per_s": world * ns / (ms * 1e-3),
                       "input_copy_ms": ms_copy,
                       "ms_excl_input_copy": ms - ms_copy,
                       "keys_per_s_excl_input_copy": world * ns / ((ms - ms_copy) * 1e-3),
                       "local_sort_ms": ms_local,
                       "bytes_model": f"{bpk:.0f} B/key",
                       "local_GBps": bpk * ns / (ms_local * 1e-3) / 1e9,
                       "frac": bpk * ns / (ms_local * 1e-3) / 1e9 / HBM_PEAK_GBS,
                       "check": check, "scaling": "weak"}
        del src, keys, ws, land
        torch.cuda.empty_cache()

    # ------------------------------------------------------------ C4 gemv
    # int64 indices: the reference's default index type (sparse_matrix<T, I =
    # std::size_t>, containers/sparse_matrix.hpp:126), 12 B per nonzero
    gemv_kinds = [(k, nm, ib) for k, nm, ib in ((0, "gemv_banded", 4), (1, "gemv", 4),
                                                (0, "gemv_banded_i64", 8), (1, "gemv_i64", 8))
                  if (ib == 4 and want("gemv")) or want(nm) or (nm == "gemv" and want("gemv_random"))]
    if gemv_kinds:
        # banded (10 diagonals, x read ~once) and random (10 uniform columns per
        # row: every nonzero gathers a separate x line) CSR, rows split over
        # ranks.  x is distributed like the rows; each call ships every rank
        # only the window of x its rows' columns span (recorded once at
        # construction: one all_gather of the column ranges), by one alltoallv
        # into a window buffer that holds the rank's own x block in place --
        # banded: +-5 neighbour elements; random: all of x (as the reference's
        # replication, gemv.hpp:30-42)
        m = 1 << args.gemv_log2m
        rows_per = (m + world - 1) // world
        row0 = min(m, rank * rows_per)
        rows = min(m, row0 + rows_per) - row0
        kk = 10
        for kind, name, ib in gemv_kinds:
            nnz = drhip.csr_nnz(kind, row0, rows, m, kk)
            with torch.cuda.stream(stream):
                rowptr = torch.empty(rows + 1, dtype=torch.int32, device="cuda")
                colind = torch.empty(max(nnz, 1), dtype=torch.int32, device="cuda")
                vals = torch.empty(max(nnz, 1), dtype=torch.float32, device="cuda")
                drhip.csr_gen(0, kind, row0, rows, m, kk, 1, rowptr.data_ptr(), colind.data_ptr(), vals.data_ptr())
                if ib == 8:  # the same matrix with 8-byte indices
                    rowptr, colind = rowptr.to(torch.int64), colind.to(torch.int64)
                    torch.cuda.empty_cache()
                y = torch.zeros(rows, dtype=torch.float32, device="cuda")
                lo, hi = (int(colind[:nnz].min().item()), int(colind[:nnz].max().item()) + 1) if nnz else (0, 0)
                s0, sl = dr_dist.x_segments(m, world)[rank]
                lo, hi = min(lo, s0), max(hi, s0 + sl)  # the window holds this rank's own x block
                wins = dr_dist.x_windows(lo, hi, torch.device("cuda"))
                plan = dr_dist.window_plan(m, wins, rank)
                xw = torch.empty(hi - lo, dtype=torch.float32, device="cuda")
                xl = xw[s0 - lo:s0 - lo + sl]  # this rank's x block, in place inside its window
                xl.copy_(torch.rand(sl, generator=torch.Generator(device="cuda").manual_seed(5 + rank), device="cuda"))
                xbase = xw.data_ptr() - 4 * lo  # x[j] at xbase + 4 j for j in the window
            win_recv = sum(plan[2]) - plan[2][rank]

            def gemv_step():
                with torch.cuda.stream(stream):
                    dr_dist.gather_x_window(xl, xw, m, wins, plan)
                    T(name, lambda: drhip.spmv_csr(0, rows, nnz, rowptr.data_ptr(), colind.data_ptr(), vals.data_ptr(),
                                                   xbase, y.data_ptr(), idtype=drhip.I32 if ib == 4 else drhip.I64))

            gemv_step()
            T.ev.clear()
            ms = timed_region(torch, dist, world, gemv_step, steps)
            ms_k = T.ms(name)
            with torch.cuda.stream(stream):  # one call from y = 0, vs fp64 rows
                y.zero_()
                gemv_step()
            torch.cuda.synchronize()
            check = check_gemv(torch, rowptr, colind, vals, dr_dist.gather_x(xl), y, nnz)
            byts = (4 + ib) * nnz + ib * (rows + 1) + 8 * rows + 4 * m
            ops[name] = {"config": f"{'banded' if kind == 0 else 'random'} CSR 2^{args.gemv_log2m} x 2^{args.gemv_log2m}, "
                                   f"~{kk} nnz/row, fp32 values, {'int32' if ib == 4 else 'int64'} indices, rows split "
                                   f"over {world} GPU(s) (C4 strong), x window exchanged every call",
                         "ms": ms, "nnz_per_s": world * nnz / (ms * 1e-3),
                         "kernel_ms": ms_k, "kernel_GBps": byts / (ms_k * 1e-3) / 1e9,
                         "frac": byts / (ms_k * 1e-3) / 1e9 / HBM_PEAK_GBS,
                         "bytes_model": ("8*nnz + 4*(m+1)" if ib == 4 else "12*nnz + 8*(m+1)") + " + 8*m + 4*n (x read once)",
                         # random columns: every gather is its own 64-byte HBM access
                         # (x does not stay in L2/MALL; tools/spmv_sweep.hip footprint probe)
                         **({"frac_gather_line_model": (byts + 60.0 * nnz) / (ms_k * 1e-3) / 1e9 / HBM_PEAK_GBS}
                            if kind == 1 else {}),
                         "check": check, "scaling": "strong"}
            ops[name]["x_exchange"] = {"window": [lo, hi], "elements_received": win_recv,
                                       "vs_full_replication": (m - sl),
                                       "note": "per call: one alltoallv of the x window (rank's own block in place)"}
            del rowptr, colind, vals, xl, xw, y
            torch.cuda.empty_cache()

    # -------------------------------------------------------- C5 stencil1d
    if want("stencil1d"):
        r = 1
        with torch.cuda.stream(stream):
            a = torch.rand(nc + 2 * r, generator=torch.Generator(device="cuda").manual_seed(9 + rank), device="cuda")
            b = torch.zeros_like(a)
        bufs = [a, b]
        lo = r if rank == 0 else 0
        hi = nc - r if rank == world - 1 else nc

        # N > 1: cells [r, nc - r) read no halo cell: computed on segment 1's
        # stream while segment 0 exchanges the halos, then the 2r edge cells
        ilo, ihi = max(lo, r), min(hi, nc - r)
        edges = [(a0, b0) for a0, b0 in ((lo, min(hi, ilo)), (max(lo, ihi), hi)) if a0 < b0]

        def stencil_step():
            if world == 1:
                with torch.cuda.stream(stream):
                    T("stencil", lambda: drhip.stencil1d(0, np.float32, bufs[0].data_ptr(), bufs[1].data_ptr(), nc, r,
                                                         lo, hi))
            else:
                def interior():
                    T1("stencil", lambda: drhip.stencil1d(1, np.float32, bufs[0].data_ptr(), bufs[1].data_ptr(), nc,
                                                          r, ilo, ihi))

                def rest():
                    dr_dist.halo_exchange(bufs[0], r)
                    for a0, b0 in edges:
                        drhip.stencil1d(0, np.float32, bufs[0].data_ptr(), bufs[1].data_ptr(), nc, r, a0, b0)
                overlap_step(torch, stream, stream1, interior, rest)
            bufs.reverse()

        stencil_step()
        T.ev.clear()
        T1.ev.clear()
        ms = timed_region(torch, dist, world, stencil_step, steps)
        ms_k = T.ms("stencil") if world == 1 else T1.ms("stencil")
        stencil_step()  # one more exchange + step, checked cell by cell
        torch.cuda.synchronize()
        src_b, out_b = bufs[1], bufs[0]  # reversed by the step
        ref = src_b[r + lo - 1:r + hi - 1] + src_b[r + lo:r + hi] + src_b[r + lo + 1:r + hi + 1]
        bad = int((ref != out_b[r + lo:r + hi]).sum().item())
        check = {"cells_checked": hi - lo, "mismatches": bad, "ok": bad == 0,
                 "ref": "torch (p[-1] + p[0]) + p[1] in fp32, bit-exact"}
        ops["stencil1d"] = {"config": f"3-point fp32, 2^{args.stencil_log2n} cells per GPU (C5 weak), halo 1 cell/side"
                                      + (", interior computed during the halo exchange" if world > 1 else ""),
                            "ms": ms, "cells_per_s": world * nc / (ms * 1e-3),
                            "kernel_ms": ms_k, "kernel_GBps": 8.0 * nc / (ms_k * 1e-3) / 1e9,
                            "frac": 8.0 * nc / (ms_k * 1e-3) / 1e9 / HBM_PEAK_GBS, "check": check,
                            "scaling": "weak"}
        del a, b, bufs, ref
        torch.cuda.empty_cache()

    # ------------------------------------------------ A5 for_each (x += 1)
    if want("for_each"):
        # in-place read-modify-write over 2^stencil_log2n fp32 cells
        with torch.cuda.stream(stream):
            a = torch.rand(nc, generator=torch.Generator(device="cuda").manual_seed(10 + rank), device="cuda")

            a0 = a.clone()
        calls = [0]

        def for_each_step():
            with torch.cuda.stream(stream):
                T("for_each", lambda: drhip.transform_scalar(0, np.float32, "plus", a.data_ptr(), a.data_ptr(), nc, 1.0))
            calls[0] += 1

        for_each_step()
        T.ev.clear()
        ms = timed_region(torch, dist, world, for_each_step, steps)
        ms_k = T.ms("for_each")
        torch.cuda.synchronize()
        for _ in range(calls[0]):
            a0 += 1.0
        bad = int((a0 != a).sum().item())
        check = {"mismatches": bad, "ok": bad == 0, "ref": f"torch x += 1 applied {calls[0]} times, bit-exact"}
        del a0
        ops["for_each"] = {"config": f"x[i] += 1 in place, fp32, 2^{args.stencil_log2n} elements per GPU (weak)",
                           "ms": ms, "elements_per_s": world * nc / (ms * 1e-3),
                           "kernel_ms": ms_k, "kernel_GBps": 8.0 * nc / (ms_k * 1e-3) / 1e9,
                           "frac": 8.0 * nc / (ms_k * 1e-3) / 1e9 / HBM_PEAK_GBS, "check": check,
                           "scaling": "weak"}
        del a
        torch.cuda.empty_cache()

    # ------------------------------------- A7 transform_reduce (dot product)
    if want("dot"):
        # reduce(zip(x, y) | transform(a*b)) (examples/shp/dot_product.cpp:11-18)
        # over 2^stencil_log2n fp32 pairs per GPU: 8 B/elem read, fp64
        # accumulation, partials folded in segment order over RCCL
        with torch.cuda.stream(stream):
            g = torch.Generator(device="cuda").manual_seed(12 + rank)
            dx = torch.rand(nc, generator=g, device="cuda")
            dy = torch.rand(nc, generator=g, device="cuda")
            dpart = torch.zeros(1, dtype=torch.float64, device="cuda")

        def dot_step():
            with torch.cuda.stream(stream):
                T("dot", lambda: drhip.dot_async(0, np.float32, dx.data_ptr(), dy.data_ptr(), nc, dpart.data_ptr()))
                dr_dist.reduce_partials(dpart, "plus")

        for _ in range(10):  # the clock ramp of a short warm-up shows in per-launch events
            dot_step()
        T.ev.clear()
        ms = timed_region(torch, dist, world, dot_step, steps)
        ms_k = T.ms("dot")
        torch.cuda.synchronize()
        ref = float(torch.dot(dx.double(), dy.double()).item())
        err = abs(float(dpart.item()) - ref) / abs(ref)
        # the same kernel on operands at different 16-byte alignments
        # (dot(x[1:], y[:-1]): y read with element loads)
        for _ in range(steps):
            with torch.cuda.stream(stream):
                T("dot_shifted", lambda: drhip.dot_async(0, np.float32, dx.data_ptr() + 4, dy.data_ptr(), nc - 1,
                                                         dpart.data_ptr()))
        torch.cuda.synchronize()
        ms_sh = T.ms("dot_shifted")
        ref_sh = float(torch.dot(dx[1:].double(), dy[:-1].double()).item())
        err_sh = abs(float(dpart.item()) - ref_sh) / abs(ref_sh)
        # the same launches back to back under ONE event pair (the A/B tool's
        # way, tools/archive/r05/dot_ab.py): per-launch event pairs vs loop timing
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(steps):
            drhip.dot_async(0, np.float32, dx.data_ptr(), dy.data_ptr(), nc, dpart.data_ptr())
        e1.record(stream)
        torch.cuda.synchronize()
        ms_loop = e0.elapsed_time(e1) / steps
        check = {"rel_err": err, "shifted_rel_err": err_sh, "tolerance": 1e-5,
                 "ok": err <= 1e-5 and err_sh <= 1e-5, "ref": "torch fp64 dot (this rank)"}
        ops["dot"] = {"config": f"transform_reduce x.y, fp32 (fp64 accumulate), 2^{args.stencil_log2n} pairs per GPU (weak)",
                      "ms": ms, "elements_per_s": world * nc / (ms * 1e-3),
                      "kernel_ms": ms_k, "kernel_GBps": 8.0 * nc / (ms_k * 1e-3) / 1e9,
                      "frac": 8.0 * nc / (ms_k * 1e-3) / 1e9 / HBM_PEAK_GBS,
                      "shifted_kernel_ms": ms_sh, "shifted_frac": 8.0 * (nc - 1) / (ms_sh * 1e-3) / 1e9 / HBM_PEAK_GBS,
                      "loop_kernel_ms": ms_loop, "loop_frac": 8.0 * nc / (ms_loop * 1e-3) / 1e9 / HBM_PEAK_GBS,
                      "y_minus_x_bytes": dy.data_ptr() - dx.data_ptr(),
                      "check": check, "scaling": "weak"}
        del dx, dy, dpart
        torch.cuda.empty_cache()

    # -------------------------------------------------------- C5 stencil2d
    if want("stencil2d"):
        # 2^16-wide rows, 2^(stencil_log2n-16) owned rows per GPU (2^16 x 2^16
        # grid at 8 GPUs), one halo row per side exchanged every step
        nx = 1 << 16
        ny = max(1, nc // nx)
        with torch.cuda.stream(stream):
            a2 = torch.rand((ny + 2) * nx, generator=torch.Generator(device="cuda").manual_seed(11 + rank), device="cuda")
            b2 = a2.clone()
        bufs2 = [a2, b2]
        rlo = 1 if rank == 0 else 0
        rhi = ny - 1 if rank == world - 1 else ny

        # N > 1: rows [1, ny - 1) read no halo row: on segment 1's stream
        # during the exchange, then the two edge rows
        irlo, irhi = max(rlo, 1), min(rhi, ny - 1)
        redges = [(a0, b0) for a0, b0 in ((rlo, min(rhi, irlo)), (max(rlo, irhi), rhi)) if a0 < b0]

        def stencil2_step():
            if world == 1:
                with torch.cuda.stream(stream):
                    T("stencil2d", lambda: drhip.stencil2d(0, np.float32, bufs2[0].data_ptr(), bufs2[1].data_ptr(), nx,
                                                           ny, rlo, rhi))
            else:
                def interior():
                    T1("stencil2d", lambda: drhip.stencil2d(1, np.float32, bufs2[0].data_ptr(), bufs2[1].data_ptr(),
                                                            nx, ny, irlo, irhi))

                def rest():
                    dr_dist.halo_exchange(bufs2[0], nx)  # one row per side
                    for a0, b0 in redges:
                        drhip.stencil2d(0, np.float32, bufs2[0].data_ptr(), bufs2[1].data_ptr(), nx, ny, a0, b0)
                overlap_step(torch, stream, stream1, interior, rest)
            bufs2.reverse()

        stencil2_step()
        T.ev.clear()
        T1.ev.clear()
        ms = timed_region(torch, dist, world, stencil2_step, steps)
        ms_k = T.ms("stencil2d") if world == 1 else T1.ms("stencil2d")
        stencil2_step()  # one more exchange + step, checked cell by cell
        torch.cuda.synchronize()
        A = bufs2[1].view(ny + 2, nx)
        Bo = bufs2[0].view(ny + 2, nx)
        c = A[1 + rlo:1 + rhi, 1:-1]
        ref = c + A[1 + rlo:1 + rhi, :-2] + A[1 + rlo:1 + rhi, 2:] + A[rlo:rhi, 1:-1] + A[2 + rlo:2 + rhi, 1:-1]
        bad = int((ref != Bo[1 + rlo:1 + rhi, 1:-1]).sum().item())
        check = {"cells_checked": int(ref.numel()), "mismatches": bad, "ok": bad == 0,
                 "ref": "torch c + w + e + n + s in fp32, bit-exact"}
        del ref, c, A, Bo
        cells = ny * nx
        ops["stencil2d"] = {"config": f"5-point fp32, {ny} x {nx} cells per GPU (C5 weak), halo 1 row/side"
                                      + (", interior rows computed during the halo exchange" if world > 1 else ""),
                            "ms": ms, "cells_per_s": world * cells / (ms * 1e-3),
                            "kernel_ms": ms_k, "kernel_GBps": 8.0 * cells / (ms_k * 1e-3) / 1e9,
                            "frac": 8.0 * cells / (ms_k * 1e-3) / 1e9 / HBM_PEAK_GBS, "check": check,
                            "scaling": "weak"}
        del a2, b2, bufs2
        torch.cuda.empty_cache()

    # ------------------- F4 dense_matrix / A5 user-lambda for_each (C++ layer)
    if want("dense") and world == 1:
        # the header-only C++ drop-in's template for_each (a user lambda, not a
        # C-ABI fixed op) over a 2^15 x 2^15 fp32 dense_matrix and a 2^30
        # distributed_vector, timed with HIP events on the segment stream by
        # tests/cpp/bin/dense_bench (one process, one device)
        import subprocess
        exe = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tests", "cpp", "bin", "dense_bench")
        if os.path.exists(exe):
            r = subprocess.run([exe, "15", "15", str(max(steps, 3))], capture_output=True, text=True, timeout=120)
            if r.returncode != 0:
                raise RuntimeError(f"dense_bench failed: {r.stdout[-500:]} {r.stderr[-500:]}")
            for line in r.stdout.splitlines():
                if line.startswith("{"):
                    d = json.loads(line)
                    ops[d.pop("op")] = d

    # every rank computed these checks on its own share: rank 0's line
    # reports ok only if it held on every rank (same ops on every rank, in
    # this fixed order, so the collectives pair up)
    for k in ("sort", "gemv_banded", "gemv", "stencil1d", "stencil2d", "for_each", "dot"):
        if k in ops and isinstance(ops[k].get("check"), dict):
            all_ranks(torch, dist, world, ops[k]["check"])

    # --------- the reference's model: ONE process driving every device
    if want("shp_one_process"):
        # tests/cpp/bin/shp_bench: shp::init({0..N-1}) through the C++ drop-in
        # (reduce, inclusive_scan, sort with cross-device piece copies), run
        # by rank 0 while the other ranks wait; weak sizes per device
        import subprocess
        exe = os.path.join(ROOT, "tests", "cpp", "bin", "shp_bench")
        if rank == 0 and os.path.exists(exe):
            torch.cuda.synchronize()
            # rank r drives device r (LOCAL_RANK); the one-GPU rehearsal maps every rank to device 0
            rehearsal = bool(os.environ.get("DRHIP_FORCE_LOCAL0"))
            devs = (",".join("0" if rehearsal else str(i) for i in range(world)) if world > 1
                    else str(torch.cuda.current_device()))
            r = subprocess.run([exe, "--devices", devs, "--log2n", str(args.log2n), "--sort-log2n",
                                str(args.sort_log2n), "--reps", "5"], capture_output=True, text=True, timeout=600)
            got = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
            if r.returncode != 0 or not got:
                ops["shp_one_process"] = {"error": (r.stdout + r.stderr)[-600:], "rc": r.returncode}
            else:
                d = json.loads(got[-1])
                ops[d.pop("op")] = d
        if world > 1:
            dist.barrier(group=CPU_GROUP)
    return ops


if __name__ == "__main__":
    sys.exit(main())
