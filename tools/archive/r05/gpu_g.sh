#!/bin/bash
# round 5, pass g: the template scan's ordered early aggregate
# (DR_SHP_LB_EARLY) -- parity with the C++ suite (non-commutative affine /
# mat2 / keep-right scans included) and three interleaved rounds of the
# lambda-op scan; then the dot grid A/B (DRHIP_DOT_BLOCKS_PER_CU 8 / 4 / 2)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for dc in 0 3 8; do
  a=""; [ $dc -gt 0 ] && a="--devicesCount $dc"
  echo "shp_tests_early1 devices $dc: $(timeout -k 10 300 tests/cpp/bin/shp_tests_early1 $a | tail -1)" || exit 1
done
for rep in 1 2 3; do
  for v in early0 early1; do
    out=$(timeout -k 10 120 tests/cpp/bin/dense_bench_$v 15 15 10) || { echo "$v failed"; exit 1; }
    echo "rep $rep $v $(echo "$out" | grep scan_lambda_op)"
  done
done
timeout -k 10 600 python3 tools/archive/r05/dot_ab.py dot8=tools/r05var/dot8/libdrhip.so dot4=tools/r05var/dot4/libdrhip.so \
  dot2=tools/r05var/dot2/libdrhip.so || exit 1
