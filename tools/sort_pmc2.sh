#!/bin/bash
# onesweep HBM counters (one counter per pass, one rocprofv3 run each) for
# the XCD-grouped (PT=1) and one-shot (PT=0) kernels, then look-back width
# variants (tools/diag/look*/libdrhip.so) timed at 2^28 u32
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
export TMPDIR=/tmp
mkdir -p gpurun_out
for pt in 1 0; do
  for c in FETCH_SIZE WRITE_SIZE; do
    rm -rf gpurun_out/spmc_${pt}_$c
    DRHIP_SORT_OS_PT=$pt timeout -s KILL 90 rocprofv3 --pmc $c -d "$R/gpurun_out/spmc_${pt}_$c" -o pmc --output-format csv \
      -- "$R/tools/sort_bench" 28 2 > gpurun_out/spmc_${pt}_$c.log 2>&1 || exit $?
  done
done
python3 - <<'PY'
import csv, glob, collections
for pt in "10":
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        f = glob.glob(f"gpurun_out/spmc_{pt}_{c}/**/*counter_collection.csv", recursive=True)
        if not f: print("no csv", pt, c); continue
        agg = collections.defaultdict(lambda: [0, 0.0])
        for r in csv.DictReader(open(f[0])):
            if "radix" not in r["Kernel_Name"]: continue
            k = r["Kernel_Name"].split("(")[0][-60:]
            agg[(k, r["Dispatch_Id"])][1] += float(r["Counter_Value"])
        per = collections.defaultdict(list)
        for (k, _), (_, v) in agg.items(): per[k].append(v)
        for k, vs in sorted(per.items()):
            print(f"PT={pt} {c:10s} {k:60s} n={len(vs):3d} raw/dispatch {sum(vs)/len(vs)*1024/1e9:8.3f} GB")
PY
for v in ${VARIANTS:-look2 look8 look16}; do
  echo "== $v"
  LD_LIBRARY_PATH=$PWD/tools/diag/$v timeout -k 10 60 ./tools/sort_bench 28 5 | grep drhip || exit 1
done
