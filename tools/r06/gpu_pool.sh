#!/bin/bash
# round 6: one discriminating pass over the pool's wrong bytes.
#  A) pool + staged copies, ScanNonCommutative with the step check (kernel
#     hash vs device-to-host copy of the input) and the allocation trace with
#     the live-overlap check (csrc/runtime.hip alloc_track)
#  B) the same with guard red zones (DRHIP_ALLOC_GUARD=1)
#  C) the standalone replay of A's traces without libdrhip (tools/pool_replay)
#  D) the default allocator, whole suite, guard on: still green
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06p
mkdir -p $O
for rep in 1 2 3 4; do
  SHP_TESTS_STEP_CHECK=1 DRHIP_ALLOC=pool DRHIP_COPY=staged DRHIP_ALLOC_TRACE=$O/trace_A$rep.txt \
    timeout -k 10 300 tests/cpp/bin/shp_tests --filter ScanNonCommutative > $O/A$rep.txt 2>&1; rc=$?
  [ $rc -ge 124 ] && { echo "A$rep rc $rc"; tail -5 $O/A$rep.txt; exit $rc; }
  echo "A$rep rc $rc: $(grep -E 'overlapping|input changed|corrupted in|FAILED' $O/A$rep.txt | head -4 | tr '\n' ' ')"
done
for rep in 1 2; do
  SHP_TESTS_STEP_CHECK=1 DRHIP_ALLOC=pool DRHIP_COPY=staged DRHIP_ALLOC_GUARD=1 DRHIP_ALLOC_TRACE=$O/trace_B$rep.txt \
    timeout -k 10 300 tests/cpp/bin/shp_tests --filter ScanNonCommutative > $O/B$rep.txt 2>&1; rc=$?
  [ $rc -ge 124 ] && { echo "B$rep rc $rc"; tail -5 $O/B$rep.txt; exit $rc; }
  echo "B$rep rc $rc: $(grep -E 'overlapping|guard|input changed|corrupted in|FAILED' $O/B$rep.txt | head -4 | tr '\n' ' ')"
done
for rep in 1 2; do
  for mode in "" "--touch" "--touch --spin-us 300"; do
    timeout -k 10 120 tools/pool_replay $O/trace_A$rep.txt $mode --reps 3 > $O/C$rep.txt 2>&1; rc=$?
    [ $rc -ge 124 ] && { echo "C$rep rc $rc"; exit $rc; }
    echo "C$rep [$mode] rc $rc: $(grep -E 'OVERLAP|replay' $O/C$rep.txt | head -3 | tr '\n' ' ')"
  done
done
DRHIP_ALLOC_GUARD=1 timeout -k 10 600 tests/cpp/bin/shp_tests > $O/D.txt 2>&1; rc=$?
echo "D rc $rc: $(grep -cE '^\[    OK' $O/D.txt) ok, $(grep -cE '^\[FAILED' $O/D.txt) failed; $(grep -E 'guard|overlapping' $O/D.txt | head -3 | tr '\n' ' ')"
for d in 1 3 8; do
  timeout -k 10 300 tests/cpp/bin/shp_tests -d $d --filter Sort > $O/E$d.txt 2>&1; rc=$?
  echo "E -d $d rc $rc: $(grep -E '^\[' $O/E$d.txt | tr '\n' ' ')"
  [ $rc -ge 124 ] && exit $rc
done
exit 0
