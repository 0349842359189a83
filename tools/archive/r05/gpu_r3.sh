#!/bin/bash
# round 5, pass r3: pool + staged copies, ScanNonCommutative with the input
# checked after every step (SHP_TESTS_STEP_CHECK): which step changes it
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for rep in $(seq 1 10); do
  SHP_TESTS_STEP_CHECK=1 DRHIP_ALLOC=pool DRHIP_COPY=staged timeout -k 10 300 tests/cpp/bin/shp_tests --filter ScanNonCommutative > gpurun_out/r3_cur.txt 2>&1; rc=$?
  [ $rc -ge 124 ] && { echo "rc $rc"; exit $rc; }
  echo "rep $rep rc $rc: $(grep -E 'input changed|right after|corrupted in| v 0x' gpurun_out/r3_cur.txt | head -4 | tr '\n' ' ')"
done
