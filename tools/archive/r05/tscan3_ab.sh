#!/bin/bash
# template scan, round-5 third A/B: head = the committed scan.hpp (DPP moves
# with an `old` operand), ilv0 = bound_ctrl DPP moves (the compiler fuses
# them into the op: v_add_f32_dpp), ilv8 = the same with the U wave scans
# interleaved in groups of 8; lambda-op scan 2^29 f32, three rounds; parity:
# the C++ suite built each way
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for b in shp_tests shp_tests_ilv8; do
  for dc in 0 8; do
    a=""; [ $dc -gt 0 ] && a="--devicesCount $dc"
    echo "$b devices $dc: $(timeout -k 10 300 tests/cpp/bin/$b $a | tail -1)" || exit 1
  done
done
for rep in 1 2 3; do
  for v in head ilv0 ilv8; do
    out=$(timeout -k 10 120 tests/cpp/bin/dense_bench_$v 15 15 10) || { echo "$v failed"; exit 1; }
    echo "rep $rep $v $(echo "$out" | grep scan_lambda_op)"
  done
done
