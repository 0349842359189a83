#!/usr/bin/env python3
"""Per-launch HBM traffic from rocprofv3 --pmc passes (measurement tool).

usage: pmc_summary.py FETCH_DIR WRITE_DIR > pmc_summary.json

FETCH_SIZE / WRITE_SIZE are KiB per dispatch (MI355X_MICROARCH.md, HBM).
gfx950 correction: FETCH_SIZE counts exactly half of the bytes of a wide
(16 B/lane) coalesced streaming read, so it is doubled; WRITE_SIZE is exact
for 16 B/lane streaming stores.  Values are averaged per kernel name.
"""
import csv
import glob
import json
import os
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
            per[name].append(float(r.get("Counter_Value") or r.get("Counter-Value")))
    return per


def main():
    fetch = load(sys.argv[1], "FETCH_SIZE")
    write = load(sys.argv[2], "WRITE_SIZE")
    out = {"note": "hbm_bytes_per_launch = (2*FETCH_SIZE + WRITE_SIZE) * 1024, averaged over "
                   "dispatches; FETCH_SIZE doubled per the gfx950 wide-read correction",
           "kernels": {}}
    for name in sorted(set(fetch) | set(write)):
        f = sum(fetch.get(name, [0])) / max(1, len(fetch.get(name, [])))
        w = sum(write.get(name, [0])) / max(1, len(write.get(name, [])))
        short = name.split("(")[0]
        out["kernels"][short] = {
            "dispatches": max(len(fetch.get(name, [])), len(write.get(name, []))),
            "fetch_kib_raw": f, "write_kib": w,
            "hbm_bytes_per_launch": (2 * f + w) * 1024.0,
        }
    json.dump(out, sys.stdout, indent=1)


if __name__ == "__main__":
    main()
