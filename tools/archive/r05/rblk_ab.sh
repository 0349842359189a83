#!/bin/bash
# round 5: template reduce grid (DRHIP_REDUCE_BLOCKS 512 / 1024 / 2048 shipped /
# 4096): dense_bench's reduce_zip_transform and reduce_lambda_op (2^29), three
# interleaved rounds
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for rep in 1 2 3; do
  for v in rb2048 rb512 rb1024 rb4096; do
    out=$(timeout -k 10 120 tests/cpp/bin/dense_bench_$v 15 15 10) || { echo "$v failed"; exit 1; }
    echo "rep $rep $v $(echo "$out" | grep -E 'reduce_zip_transform|reduce_lambda_op' | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['op'], d['ms'], d['frac'], d.get('check'), end='  ')")"
  done
done
