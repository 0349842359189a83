#!/bin/bash
# template (user-operator) scan variants, tests/cpp/bin/dense_bench_b<BUF>p<PUB>f<FAST>
# (DR_SHP_LB_BUF / _PUB / _FAST, include/dr/shp/scan.hpp): 2^29 f32 lambda-op
# scan, three interleaved rounds
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for rep in 1 2 3; do
  for v in b0p0f0 b1p0f0 b1p1f0 b1p1f1 b0p0f1; do
    out=$(timeout -k 10 120 tests/cpp/bin/dense_bench_$v 15 15 10) || { echo "$v failed"; exit 1; }
    echo "rep $rep $v $(echo "$out" | grep scan_lambda_op)"
  done
done
