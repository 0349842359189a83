#!/bin/bash
# onesweep 4-byte vs 8-byte status words; sort parity
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_sort.py -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/pytest_sort.log 2>&1
rc=$?; tail -n 2 gpurun_out/pytest_sort.log; [ $rc -eq 0 ] || exit $rc
for w in w32 w64; do
  echo "== $w"; DRHIP_SORT_STATUS=$w timeout -k 10 60 ./tools/sort_bench 28 5 | head -n 1 || exit $?
done
