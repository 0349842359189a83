#!/bin/bash
# round 5, pass o: which pool setting returns zero pages.  The C++ suite
# (shp_tests, 1 segment) NREP times per allocator variant, interleaved, with
# pageable copies staged through pinned memory (DRHIP_COPY=staged, the
# strongest amplifier): A = default pool, B = a private pool
# (hipMemPoolCreate), C = default pool without cross-stream / opportunistic
# reuse, D = hipMalloc (the shipped default)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
declare -A nf
V="A B C D"
for rep in $(seq 1 ${NREP:-30}); do
  for v in $V; do
    case $v in
      A) env="DRHIP_ALLOC=pool" ;;
      B) env="DRHIP_ALLOC=pool DRHIP_POOL=private" ;;
      C) env="DRHIP_ALLOC=pool DRHIP_POOL=noreuse" ;;
      D) env="" ;;
    esac
    env DRHIP_COPY=staged $env timeout -k 10 300 tests/cpp/bin/shp_tests > gpurun_out/o_$v.txt 2>&1; rc=$?
    [ $rc -ge 124 ] && { echo "$v rc $rc"; tail -5 gpurun_out/o_$v.txt; exit $rc; }
    if [ $rc -ne 0 ]; then nf[$v]=$(( ${nf[$v]:-0} + 1 )); [ ${nf[$v]} -le 2 ] && { echo "rep $rep $v FAILED:"; grep -E "FAILED|corrupted|right after|exception" gpurun_out/o_$v.txt | head -6; }; fi
  done
  [ $((rep % 10)) -eq 0 ] && echo "rep $rep done"
done
for v in $V; do echo "failures: $v ${nf[$v]:-0} / ${NREP:-30}"; done
