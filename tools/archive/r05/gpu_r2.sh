#!/bin/bash
# round 5, pass r2: the pool corruption without any scan (allocation, zero
# fill, staged copy, read-back, free only: SHP_TESTS_NO_SCAN), 10 runs each
# on the pool and on hipMalloc
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for alloc in pool hipmalloc; do
  nf=0
  for rep in $(seq 1 10); do
    SHP_TESTS_NO_SCAN=1 DRHIP_ALLOC=$alloc DRHIP_COPY=staged timeout -k 10 300 tests/cpp/bin/shp_tests --filter ScanNonCommutative > gpurun_out/r2_cur.txt 2>&1; rc=$?
    [ $rc -ge 124 ] && { echo "rc $rc"; exit $rc; }
    [ $rc -ne 0 ] && nf=$((nf+1))
  done
  echo "no-scan $alloc: $nf of 10 failed; last: $(grep -E 'right after|FAILED|tests,' gpurun_out/r2_cur.txt | tr '\n' ' ')"
done
