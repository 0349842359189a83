#!/usr/bin/env python3
"""Per-launch HBM traffic from rocprofv3 --pmc passes (measurement tool).

usage: pmc_summary.py FETCH_DIR WRITE_DIR > pmc_summary.json
       pmc_summary.py --calib OUT_DIR     > pmc_calib_summary.json

FETCH_SIZE / WRITE_SIZE are KiB per dispatch (MI355X_MICROARCH.md, HBM).
Raw counter values are reported per kernel, averaged over dispatches; no
blanket correction is applied.  The guide's gfx950 factor (FETCH_SIZE = 1/2
of the bytes of a 16-B/lane streaming read) holds for wide streaming reads
only; `--calib` measures the factor for every access class the kernels use
(tools/pmc_calib.hip: 16-B and 4-B streams, 4-B gathers on distinct 128-B /
64-B lines, 4-B scattered stores, 16-B stores) and reports the C4 SpMV (one
bench run per matrix kind) and the sort kernels next to them.
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def load(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True)
    per = defaultdict(list)
    for f in files:
        for r in csv.DictReader(open(f)):
            name = r.get("Kernel_Name") or r.get("Kernel-Name") or ""
            cn = r.get("Counter_Name") or r.get("Counter-Name")
            if cn != counter:
                continue
            per[name.split("(")[0]].append(float(r.get("Counter_Value") or r.get("Counter-Value")))
    return per


def avg(v):
    return sum(v) / len(v) if v else None


# Kernels whose reads are all 16-B/lane coalesced streams: the guide's
# calibrated x2 FETCH_SIZE factor applies (confirmed by cal_read16 in --calib).
STREAM16 = ("reduce_stage1", "reduce_tiles_kernel", "scan_kernel", "scan_given", "scan_wave_given", "unary_kernel",
            "binary_kernel", "dot_kernel", "dot_stage1")


def per_kernel(fetch, write):
    out = {}
    for name in sorted(set(fetch) | set(write)):
        f, w = avg(fetch.get(name, [])), avg(write.get(name, []))
        out[name] = {"dispatches": max(len(fetch.get(name, [])), len(write.get(name, []))),
                     "fetch_bytes_raw": None if f is None else f * 1024.0,
                     "write_bytes_raw": None if w is None else w * 1024.0}
        if f is not None and w is not None and any(k in name for k in STREAM16):
            out[name]["hbm_bytes_per_launch"] = (2 * f + w) * 1024.0
    return out


def calib(d):
    known = {}
    for line in open(os.path.join(d, "calib_time.log")):
        m = re.match(r"(\S+)\s+launches (\d+) avg_ms ([\d.]+) known ([\d.e+]+) (.*)", line.strip())
        if m:
            known[m.group(1)] = {"avg_ms": float(m.group(3)), "known": float(m.group(4)), "unit": m.group(5)}
    ker = per_kernel(load(os.path.join(d, "calib_FETCH_SIZE"), "FETCH_SIZE"),
                     load(os.path.join(d, "calib_WRITE_SIZE"), "WRITE_SIZE"))
    table = {}
    for name, k in known.items():
        c = ker.get(name, {})
        f, w = c.get("fetch_bytes_raw"), c.get("write_bytes_raw")
        row = dict(k)
        if f is not None:
            row["fetch_raw_per_known"] = f / k["known"]
        if w is not None:
            row["write_raw_per_known"] = w / k["known"]
        table[name] = row
    ops = {}
    for op in ("gemv_banded", "gemv_random", "sort"):
        fd, wd = os.path.join(d, f"pmc_{op}_FETCH_SIZE"), os.path.join(d, f"pmc_{op}_WRITE_SIZE")
        if os.path.isdir(fd):
            ops[op] = per_kernel(load(fd, "FETCH_SIZE"), load(wd, "WRITE_SIZE"))
    return {"note": "raw = counter KiB x 1024 per dispatch, no correction; calibration rows divide by "
                    "the kernel's known bytes (or known accesses)", "calibration": table, "ops": ops}


def main():
    if sys.argv[1] == "--calib":
        json.dump(calib(sys.argv[2]), sys.stdout, indent=1)
        return
    if sys.argv[1] == "--current":
        # --current SUMMARY COMMIT: profiles/pmc_current.json names SUMMARY
        # (a file under profiles/) as the PMC pass of the code at COMMIT;
        # bench.py reads roofline.traffic from it and records both
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        name, commit = sys.argv[2], sys.argv[3]
        if not os.path.exists(os.path.join(root, "profiles", name)):
            sys.exit(f"profiles/{name} does not exist")
        with open(os.path.join(root, "profiles", "pmc_current.json"), "w") as f:
            json.dump({"file": name, "commit": commit,
                       "note": "the PMC summary bench.py reports as roofline.traffic; rewritten with every new "
                               "PMC pass (tools/pmc_summary.py --current)"}, f)
        return
    json.dump({"note": "raw = counter KiB x 1024 per dispatch, no correction (see --calib)",
               "kernels": per_kernel(load(sys.argv[1], "FETCH_SIZE"), load(sys.argv[2], "WRITE_SIZE"))},
              sys.stdout, indent=1)


if __name__ == "__main__":
    main()
