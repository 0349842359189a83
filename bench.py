#!/usr/bin/env python3
"""bench.py -- Distributed Ranges shp hot path on MI355X.

Workload (BASELINE.json configs[1]): one STEP = shp::reduce + shp::inclusive_scan
(plus) over a distributed_vector<float> of 2^30 elements PER GPU (weak
scaling), inputs resident in HBM.  One process per GPU (torch.distributed.run
for N > 1); each rank owns one segment and calls libdrhip.so through its
C-ABI (distributed-ranges_amd/drhip.py).  Cross-segment combines run over
RCCL (torch.distributed "nccl" backend):
  reduce: local drhip_reduce -> all_gather of the N fp64 partials -> fold in
          segment order (shp/algorithms/reduce.hpp:81-83);
  scan:   local drhip_reduce of the segment total -> all_gather -> exclusive
          prefix of the preceding totals in fp64 on the device -> ONE
          single-pass drhip_inclusive_scan with that carry read by the kernel
          (carry_dev).  At N = 1 the scan is the single pass alone.

Prints ONE JSON line (rank 0).  `value` = elements of the distributed vector
processed per second by the whole job (N * 2^30 / step time).  `roofline` is
for the dominant kernel (the scan): algorithmic bytes 8 B/elem x elements per
launch / mean launch time from HIP events on the drhip stream.
`cpu_baseline` times the oracle's restatement of the reference mhp CPU path
(oracle/liboracle.so: per-rank std::reduce + gather, 3-phase scan) on the
host cores, rank 0 only, on a bounded sample.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "distributed-ranges_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X spec, MI355X_MICROARCH.md chip table


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--log2n", type=int, default=30, help="elements per GPU = 2^log2n")
    p.add_argument("--dtype", default="f32", choices=["f32", "i32"])
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=12.0)
    return p.parse_args()


def load_pmc(kernel_substr):
    """Per-launch HBM bytes of a kernel from profiles/pmc_summary.json
    (written by tools/pmc_summary.py from rocprofv3 --pmc runs, FETCH_SIZE
    doubled per the gfx950 correction)."""
    path = os.path.join(ROOT, "profiles", "pmc_summary.json")
    if not os.path.exists(path):
        return None
    try:
        d = json.load(open(path))
        for name, v in d.get("kernels", {}).items():
            if kernel_substr in name:
                return v.get("hbm_bytes_per_launch")
    except Exception:
        return None
    return None


def cpu_baseline(n_gpu_elems, seconds, dtype):
    """Oracle restatement of the reference's mhp CPU path (reduce + 3-phase
    scan), nthreads = host share, bounded sample."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    cores = min(16, os.cpu_count() or 1)
    n = 1 << 27
    rng = np.random.default_rng(1)
    if dtype == "f32":
        x = rng.random(n, dtype=np.float32)
    else:
        x = rng.integers(0, 1 << 16, n, dtype=np.int32)
    out = np.empty_like(x)
    reps = 0
    t0 = time.perf_counter()
    while True:
        if dtype == "f32":
            O.mhp_reduce_f32(x, cores, 0.0, cores)
        else:
            O.mhp_reduce_i32(x, cores, 0, cores)
        O.mhp_scan(x, cores, cores, out=out)
        reps += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    return {"value": n * reps / el, "unit": "elements/s", "cores": cores, "kind": "port",
            "sample": f"{reps} x (mhp reduce + 3-phase scan) over 2^27 {dtype} on {cores} "
                      f"OpenMP ranks/threads ({el:.1f} s); oracle/liboracle.so"}


def main():
    args = parse()
    import torch
    import torch.distributed as dist
    import drhip

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            print("for --gpus N > 1 launch with torch.distributed.run", file=sys.stderr)
            return 2
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    drhip.init([local])  # this rank's segment: one per GPU
    stream = torch.cuda.ExternalStream(drhip.stream(0))
    n = 1 << args.log2n
    np_dt = {"f32": "float32", "i32": "int32"}[args.dtype]
    tdt = {"f32": torch.float32, "i32": torch.int32}[args.dtype]
    acc_t = torch.float64 if args.dtype == "f32" else torch.int32
    import numpy as np
    dt_np = np.dtype(np_dt)

    with torch.cuda.stream(stream):
        g = torch.Generator(device="cuda").manual_seed(1 + rank)
        if args.dtype == "f32":
            x = torch.rand(n, generator=g, device="cuda", dtype=tdt)
        else:
            x = torch.randint(0, 1 << 16, (n,), generator=g, device="cuda", dtype=tdt)
        out = torch.empty_like(x)
        red_part = torch.zeros(1, dtype=acc_t, device="cuda")
        scan_tot = torch.zeros(1, dtype=acc_t, device="cuda")
        gathered_r = torch.zeros(world, dtype=acc_t, device="cuda")
        gathered_s = torch.zeros(world, dtype=acc_t, device="cuda")
        carry = torch.zeros(1, dtype=acc_t, device="cuda")
        result = torch.zeros(1, dtype=acc_t, device="cuda")
    torch.cuda.synchronize()

    ev = {k: [] for k in ("reduce", "scan")}

    def step(record):
        with torch.cuda.stream(stream):
            e0 = torch.cuda.Event(enable_timing=True) if record else None
            e1 = torch.cuda.Event(enable_timing=True) if record else None
            e2 = torch.cuda.Event(enable_timing=True) if record else None
            e3 = torch.cuda.Event(enable_timing=True) if record else None
            # ---- shp::reduce
            if record:
                e0.record(stream)
            drhip.reduce_async(0, dt_np, "plus", x.data_ptr(), n, red_part.data_ptr())
            if record:
                e1.record(stream)
            if world > 1:
                dist.all_gather_into_tensor(gathered_r, red_part)
                torch.sum(gathered_r, 0, keepdim=True, out=result)
            # ---- shp::inclusive_scan
            carry_ptr = None
            if world > 1:
                drhip.reduce_async(0, dt_np, "plus", x.data_ptr(), n, scan_tot.data_ptr())
                dist.all_gather_into_tensor(gathered_s, scan_tot)
                if rank > 0:
                    torch.sum(gathered_s[:rank], 0, keepdim=True, out=carry)
                    carry_ptr = carry.data_ptr()
            if record:
                e2.record(stream)
            drhip.scan_async(0, dt_np, "plus", x.data_ptr(), out.data_ptr(), n, carry_dev=carry_ptr)
            if record:
                e3.record(stream)
                ev["reduce"].append((e0, e1))
                ev["scan"].append((e2, e3))

    for _ in range(args.warmup):
        step(False)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    drhip.sync(0)  # surfaces an in-kernel timeout, if any

    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())

    ms_red = sum(a.elapsed_time(b) for a, b in ev["reduce"]) / len(ev["reduce"])
    ms_scan = sum(a.elapsed_time(b) for a, b in ev["scan"]) / len(ev["scan"])
    isz = dt_np.itemsize

    # sanity (outside the timed region): last scanned element equals the
    # running total through this segment
    with torch.cuda.stream(stream):
        drhip.reduce_async(0, dt_np, "plus", x.data_ptr(), n, red_part.data_ptr())
    torch.cuda.synchronize()
    seg_total = float(red_part.item())
    expect_last = seg_total + (float(carry.item()) if (world > 1 and rank > 0) else 0.0)
    last = float(out[-1].item())
    rel = abs(last - expect_last) / max(abs(expect_last), 1e-30)

    scan_bytes = 2 * isz * n
    achieved = scan_bytes / (ms_scan * 1e-3) / 1e9
    traffic = load_pmc("scan_kernel")
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
        "config": {"workload": f"shp reduce + inclusive_scan (plus), distributed_vector<{ 'float' if args.dtype == 'f32' else 'int32'}> "
                               f"2^{args.log2n} elements per GPU, one segment per GPU",
                   "elements_per_gpu": n, "global_elements": world * n,
                   "parallelism": f"segments{world}", "combine": "rccl all_gather" if world > 1 else "none"},
        "roofline": {"bound": "hbm", "kernel": "drhip::scan_kernel (single-pass decoupled look-back)",
                     "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS,
                     "traffic": traffic,
                     "algorithmic_bytes_per_launch": scan_bytes,
                     "launch_ms": ms_scan},
        "ops": {
            "reduce": {"ms": ms_red, "elements_per_s": n / (ms_red * 1e-3),
                       "GBps": isz * n / (ms_red * 1e-3) / 1e9,
                       "frac": isz * n / (ms_red * 1e-3) / 1e9 / HBM_PEAK_GBS,
                       "traffic": load_pmc("reduce_stage1")},
            "inclusive_scan": {"ms": ms_scan, "elements_per_s": n / (ms_scan * 1e-3), "GBps": achieved,
                               "frac": achieved / HBM_PEAK_GBS},
        },
        "check": {"scan_last_vs_reduce_rel": rel},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        res["cpu_baseline"] = cpu_baseline(n, args.cpu_seconds, args.dtype)
    elif rank == 0:
        res["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(res), flush=True)
    drhip.finalize()
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
