#!/bin/bash
# round 5, pass h: (1) the NT=512 group rows of profiles/r04_sort_nt_ab.txt
# re-run as the corrected tools/archive/gpu_r04_f.sh states them (DRHIP_SORT_OS_NT=512
# set), interleaved with the 256-thread default; (2) rocprofv3 kernel stats of
# dense_bench (the template scan's kernel time against its blocking-call time)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2 3; do
  for cfg in "512 16" "512 64" "256 64"; do
    set -- $cfg
    out=$(DRHIP_SORT_OS_NT=$1 DRHIP_SORT_OS_GROUP=$2 timeout -k 10 60 ./tools/sort_bench 28 5) || { echo "sort_bench NT=$1 G=$2 failed"; exit 1; }
    echo "rep $rep NT=$1 group $2: $(echo "$out" | grep drhip)"
  done
done
timeout -k 10 120 tests/cpp/bin/dense_bench 15 15 10 || exit 1
rm -rf gpurun_out/r05h_dense_prof
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/r05h_dense_prof" -o run --output-format csv \
  -- tests/cpp/bin/dense_bench 15 15 10 > gpurun_out/r05h_dense_prof.log 2>&1 || exit $?
f=$(find gpurun_out/r05h_dense_prof -name '*kernel_stats.csv' | head -1)
cut -c1-220 "$f"
