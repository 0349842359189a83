#!/bin/bash
# round 5, pass m: 25 whole-suite runs of the default build and of e0 at one
# segment, interleaved (the intermittent ScanNonCommutative failure of pass j)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
declare -A nf
for rep in $(seq 1 ${NREP:-25}); do
  for v in ${VARIANTS:-shp_tests shp_tests_e0}; do
    timeout -k 10 300 tests/cpp/bin/$v > gpurun_out/m_$v.txt 2>&1; rc=$?
    [ $rc -ge 124 ] && { echo "$v rc $rc"; exit $rc; }
    if [ $rc -ne 0 ]; then nf[$v]=$(( ${nf[$v]:-0} + 1 )); echo "rep $rep $v FAILED: $(grep -E 'failed|FAILED|noncommutative_case|exception|corrupted| v 0x|right after' gpurun_out/m_$v.txt | head -8 | tr '\n' ' ')"; cp gpurun_out/m_$v.txt gpurun_out/m_${v}_fail_$rep.txt; fi
  done
  [ $((rep % 10)) -eq 0 ] && echo "rep $rep done"
done
for v in ${VARIANTS:-shp_tests shp_tests_e0}; do echo "failures: $v ${nf[$v]:-0} / ${NREP:-25}"; done
