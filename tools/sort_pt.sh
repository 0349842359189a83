#!/bin/bash
# persistent vs one-shot onesweep: timing at 2^28 and 2^26 u32, per-kernel
# stats of each, then the sort parity tests
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for pt in 1 0; do
  echo "== DRHIP_SORT_OS_PT=$pt"
  DRHIP_SORT_OS_PT=$pt timeout -k 10 60 ./tools/sort_bench 28 5 || exit $?
  DRHIP_SORT_OS_PT=$pt timeout -k 10 60 ./tools/sort_bench 26 5 || exit $?
  rm -rf gpurun_out/sortprof$pt
  DRHIP_SORT_OS_PT=$pt timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/sortprof$pt" -o run \
    --output-format csv -- ./tools/sort_bench 28 3 > gpurun_out/sortprof$pt.log 2>&1 || exit $?
  python3 - "$pt" <<'PY'
import csv, glob, sys
f = glob.glob(f"gpurun_out/sortprof{sys.argv[1]}/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "radix" in r["Name"]:
        print(f'{r["Name"][:70]:70s} {r["Calls"]:>4s} {float(r["AverageNs"])/1e3:8.1f} us')
PY
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_sort.py -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/pytest_sort.log 2>&1
rc=$?; tail -n 3 gpurun_out/pytest_sort.log; exit $rc
