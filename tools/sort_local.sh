#!/bin/bash
# same-XCD status copy on/off: timing + per-kernel stats, then sort parity
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for l in 1 0 1 0; do
  echo "== DRHIP_SORT_OS_LOCAL=$l"
  DRHIP_SORT_OS_LOCAL=$l timeout -k 10 60 ./tools/sort_bench 28 5 | grep drhip || exit 1
done
rm -rf gpurun_out/sortprofL
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/sortprofL" -o run --output-format csv \
  -- ./tools/sort_bench 28 3 > gpurun_out/sortprofL.log 2>&1 || exit $?
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/sortprofL/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "radix" in r["Name"]:
        print(f'{r["Name"][:70]:70s} {r["Calls"]:>4s} {float(r["AverageNs"])/1e3:8.1f} us')
PY
bash tools/sort_parity.sh
