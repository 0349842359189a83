#!/bin/bash
# sort measurements: parity tests (every path), classic vs onesweep shapes, kernel trace
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_sort.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/sort_tests.log 2>&1; rc=$?; tail -2 gpurun_out/sort_tests.log; [ $rc -eq 0 ] || exit $rc
for l in ${SORT_LOG2N:-24 26 28}; do
  for a in "DRHIP_SORT_ALGO=classic" "DRHIP_SORT_ALGO=onesweep"; do
    echo "== $a 2^$l"
    env $a timeout -k 10 60 ./tools/sort_bench $l 5 > gpurun_out/sb.txt || exit $?
    head -1 gpurun_out/sb.txt
  done
done
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/sortprof" -o run --output-format csv -- "$R/tools/sort_bench" 28 3 > gpurun_out/sortprof.log 2>&1 || exit $?
