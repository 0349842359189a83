#!/bin/bash
# round 4: onesweep 512-thread (32 K-key) tiles vs 256-thread (16 K-key):
# interleaved timing, per-kernel stats of both, then sort parity on the default
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for nt in 512 256 512 256 512 256; do
  echo "== DRHIP_SORT_OS_NT=$nt"
  DRHIP_SORT_OS_NT=$nt timeout -k 10 60 ./tools/sort_bench 28 5 | grep drhip || exit 1
done
for g in 16 64; do
  echo "== NT=512 group $g"
  DRHIP_SORT_OS_NT=512 DRHIP_SORT_OS_GROUP=$g timeout -k 10 60 ./tools/sort_bench 28 5 | grep drhip || exit 1
done
for nt in 512 256; do
  rm -rf gpurun_out/sortprof_nt$nt
  DRHIP_SORT_OS_NT=$nt timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/sortprof_nt$nt" -o run --output-format csv \
    -- ./tools/sort_bench 28 3 > gpurun_out/sortprof_nt$nt.log 2>&1 || exit $?
done
python3 - <<'PY'
import csv, glob
for nt in (512, 256):
    f = glob.glob(f"gpurun_out/sortprof_nt{nt}/**/*kernel_stats.csv", recursive=True)[0]
    print("NT", nt)
    for r in csv.DictReader(open(f)):
        if "radix" in r["Name"]:
            print(f'  {r["Name"][:90]:90s} {r["Calls"]:>4s} {float(r["AverageNs"])/1e3:8.1f} us')
PY
bash tools/sort_parity.sh
