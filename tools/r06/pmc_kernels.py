#!/usr/bin/env python3
"""Per-kernel averages of every counter in rocprofv3 --pmc CSV passes
(measurement tool): {kernel: {counter: mean per dispatch, "dispatches": n}}.
usage: pmc_kernels.py PASS_DIR ... > summary.json"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main():
    acc = defaultdict(lambda: defaultdict(list))
    for d in sys.argv[1:]:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                name = (r.get("Kernel_Name") or r.get("Kernel-Name") or "").split("(")[0]
                cn = r.get("Counter_Name") or r.get("Counter-Name")
                v = r.get("Counter_Value") or r.get("Counter-Value")
                if cn and v is not None:
                    acc[name][cn].append(float(v))
    out = {}
    for k, cs in acc.items():
        out[k] = {c: sum(v) / len(v) for c, v in cs.items()}
        out[k]["dispatches"] = max(len(v) for v in cs.values())
    json.dump(out, sys.stdout, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
