#!/bin/bash
# round 5, pass n: epoch statuses (ep) against the per-call reset (e0) on the
# hipMalloc allocator, TEXC on in both: the C++ suite at 0 / 3 / 8 segments
# for both builds, then four interleaved dense_bench rounds
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for b in shp_tests shp_tests_ep; do
  for dc in 0 3 8; do
    a=""; [ $dc -gt 0 ] && a="--devicesCount $dc"
    out=$(timeout -k 10 300 tests/cpp/bin/$b $a) || { echo "$b devices $dc FAILED"; echo "$out" | grep -E "failed|FAILED|exception|noncommutative" | head -20; exit 1; }
    echo "$b devices $dc: $(echo "$out" | tail -1)"
  done
done
for rep in 1 2 3 4; do
  for v in e0 ep; do
    out=$(timeout -k 10 120 tests/cpp/bin/dense_bench_$v 15 15 10) || { echo "$v failed"; exit 1; }
    echo "rep $rep $v $(echo "$out" | grep scan_lambda_op)"
  done
done
