#!/bin/bash
# round 6, pass w: per-kernel times of the sort per key distribution (rocprofv3 kernel stats)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06w
mkdir -p $O
for k in u32 u16 f32rand f32randn; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$k -o s --output-format csv -- python3 tools/r06/sort_case.py $k > $O/prof_$k.log 2>&1 || exit 1
  python3 - <<PY
import csv
rows = [r for r in csv.DictReader(open("$O/prof_$k/s_kernel_stats.csv")) if "radix" in r["Name"]]
print("$k", "  ".join("%s %.3f" % (r["Name"].split("(")[0].replace("void drhip::", "")[:40], float(r["AverageNs"]) / 1e6) for r in rows))
PY
done
