#!/bin/bash
# SQ counters of the radix sort kernels (measurement only): where the
# scatter's wave cycles go.  One pass, 8 SQ counters.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
rm -rf gpurun_out/sort_pmc
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT \
  -d "$PWD/gpurun_out/sort_pmc" -o pmc --output-format csv -- "$PWD/tools/sort_bench" 28 2 > gpurun_out/sort_pmc.log 2>&1 || exit $?
python3 - <<'PY'
import csv, glob, collections
f = glob.glob("gpurun_out/sort_pmc/**/*counter_collection.csv", recursive=True)[0]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
n = collections.Counter()
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"][:60]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    if r["Counter_Name"] == "SQ_WAVE_CYCLES":
        n[k] += 1
for k, v in agg.items():
    w = v["SQ_WAVE_CYCLES"] or 1
    print(k, "disp", n[k], " ".join(f"{c.replace('SQ_','')}={v[c]/w:.3f}" for c in sorted(v) if c != "SQ_WAVE_CYCLES"))
PY
