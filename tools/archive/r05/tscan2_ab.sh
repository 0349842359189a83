#!/bin/bash
# template scan, round-5 second A/B: nv1 = the default (1 x 16-B vector per
# lane per slot, U = 32, 2 waves/SIMD), nv2 (2 adjacent vectors per slot,
# U = 17), u24w3 (U = 24 at 3 waves/SIMD), nv2w3 (2 vectors, U = 15, 3
# waves/SIMD): lambda-op scan 2^29 f32, three interleaved rounds; parity of
# nv2 with the C++ suite
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for dc in 0 8; do
  a=""; [ $dc -gt 0 ] && a="--devicesCount $dc"
  echo "shp_tests_nv2 devices $dc: $(timeout -k 10 300 tests/cpp/bin/shp_tests_nv2 $a | tail -1)" || exit 1
done
for rep in 1 2 3; do
  for v in nv1 nv2 u24w3 nv2w3; do
    out=$(timeout -k 10 120 tests/cpp/bin/dense_bench_$v 15 15 10) || { echo "$v failed"; exit 1; }
    echo "rep $rep $v $(echo "$out" | grep scan_lambda_op)"
  done
done
