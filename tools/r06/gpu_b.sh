#!/bin/bash
# round 6, pass b: (1) the standalone reproducer (tools/pool_tlb_repro, no
# libdrhip) on pass a's allocation traces, pool and hipMalloc; (2) the
# caching allocator (DRHIP_ALLOC=cache) under the configuration that failed
# 28-30 of 30 runs with the pool (staged copies), step check and guard on;
# (3) the allocators' price (shp_bench --overhead); (4) the C++ suite with
# guard red zones on the default allocator; (5) C4 through the drop-in
# (sparse_matrix<float, size_t>, shp::gemv) at 2^26 over 8 segments; (6) C5
# through dr/mhp.hpp at 2^32 over 8 MPI ranks.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06b
mkdir -p $O
for t in A1 A3 A4; do
  for a in pool hipmalloc; do
    timeout -k 10 180 tools/pool_tlb_repro gpurun_out/r06p/trace_$t.txt --alloc $a --reps 3 > $O/repro_${t}_$a.txt 2>&1; rc=$?
    echo "repro $t $a rc $rc: $(tail -1 $O/repro_${t}_$a.txt) | $(grep -m3 WRONG $O/repro_${t}_$a.txt | tr '\n' ' ')"
    [ $rc -ge 124 ] && exit $rc
  done
done
for rep in 1 2 3 4 5; do
  SHP_TESTS_STEP_CHECK=1 DRHIP_ALLOC=cache DRHIP_COPY=staged DRHIP_ALLOC_GUARD=1 timeout -k 10 600 tests/cpp/bin/shp_tests > $O/cache_$rep.txt 2>&1; rc=$?
  echo "cache+staged rep $rep rc $rc: $(grep -cE '^\[    OK' $O/cache_$rep.txt) ok, $(grep -cE '^\[FAILED' $O/cache_$rep.txt) failed; $(grep -E 'guard|overlapping|input changed' $O/cache_$rep.txt | head -3 | tr '\n' ' ')"
  [ $rc -ge 124 ] && exit $rc
done
for a in hipmalloc cache pool; do
  DRHIP_ALLOC=$a timeout -k 10 120 tests/cpp/bin/shp_bench --overhead 0 > $O/price_$a.txt 2>&1; rc=$?
  echo "price $a rc $rc: $(grep alloc_price $O/price_$a.txt)"
  [ $rc -ge 124 ] && exit $rc
done
DRHIP_ALLOC_GUARD=1 timeout -k 10 600 tests/cpp/bin/shp_tests > $O/guard_default.txt 2>&1; rc=$?
echo "guard default rc $rc: $(grep -cE '^\[    OK' $O/guard_default.txt) ok, $(grep -cE '^\[FAILED' $O/guard_default.txt) failed; $(grep -E 'guard|overlapping' $O/guard_default.txt | head -3 | tr '\n' ' ')"
[ $rc -ge 124 ] && exit $rc
for k in banded random; do
  timeout -k 10 400 tests/cpp/bin/config_tests c4 26 8 --kind $k --index i64 > $O/c4_$k.txt 2>&1; rc=$?
  echo "c4 $k rc $rc: $(grep '^{' $O/c4_$k.txt)"
  [ $rc -ge 124 ] && exit $rc
done
timeout -k 10 600 /opt/conda/bin/mpiexec -n 8 tests/cpp/bin/mhp_tests_mpi --transport mpi --c5 32 3 > $O/c5.txt 2>&1; rc=$?
echo "c5 rc $rc: $(grep '^{' $O/c5.txt) $(tail -3 $O/c5.txt | tr '\n' ' ')"
exit 0
