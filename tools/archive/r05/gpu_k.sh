#!/bin/bash
# round 5, pass k: bisect the ScanNonCommutative failure of pass j
# (default = epoch statuses + layout rule; nolc = epoch statuses without the
# layout rule; e0 = the per-call reset)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for v in shp_tests shp_tests_nolc shp_tests_e0; do
  for rep in 1 2 3; do
    timeout -k 10 300 tests/cpp/bin/$v --filter ScanNonCommutative > gpurun_out/k_$v.txt 2>&1; rc=$?
    [ $rc -ge 124 ] && { echo "$v rc $rc"; cat gpurun_out/k_$v.txt; exit $rc; }
    echo "$v rep $rep rc $rc: $(grep -E 'noncommutative_case|tests,' gpurun_out/k_$v.txt | head -3 | tr '\n' ' ')"
  done
  timeout -k 10 300 tests/cpp/bin/$v > gpurun_out/k_$v.txt 2>&1; rc=$?
  [ $rc -ge 124 ] && { echo "$v rc $rc"; exit $rc; }
  echo "$v full rc $rc: $(grep -E 'FAILED|noncommutative_case|tests,' gpurun_out/k_$v.txt | head -6 | tr '\n' ' ')"
done
