#!/bin/bash
# classic (histogram + scatter per pass) vs onesweep with the atomic ranking
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for a in classic onesweep; do
  echo "== $a"
  DRHIP_SORT_ALGO=$a timeout -k 10 60 ./tools/sort_bench 28 5 | head -n 1 || exit $?
  rm -rf gpurun_out/sortprof_$a
  DRHIP_SORT_ALGO=$a timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/sortprof_$a" -o run --output-format csv \
    -- ./tools/sort_bench 28 3 > gpurun_out/sortprof_$a.log 2>&1 || exit $?
done
