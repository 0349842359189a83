#!/bin/bash
# for_each over non-staged accessors (enumerate = zip(iota, span): a write of
# every element) with E = 1 / 4 consecutive elements per thread per step
# (DRHIP_FOREACH_BLK): dense_bench's enumerate and zip ops, three rounds
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for rep in 1 2 3; do
  for v in blk1 blk4; do
    out=$(timeout -k 10 120 tests/cpp/bin/dense_bench_$v 15 15 10) || { echo "$v failed"; exit 1; }
    echo "rep $rep $v $(echo "$out" | grep -E 'enumerate_for_each|dense_for_each' | tr '\n' ' ')"
  done
done
