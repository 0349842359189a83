#!/bin/bash
# sort parity (every algo/rank mode), timing vs rocPRIM, per-tile stamps
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_sort.py -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/pytest_sort.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_sort.log; [ $rc -eq 0 ] || exit $rc
for r in atomic ballot; do
  echo "== rank $r"
  DRHIP_SORT_RANK=$r timeout -k 10 60 ./tools/sort_bench 28 5 || exit $?
  DRHIP_SORT_RANK=$r DRHIP_SORT_ALGO=classic timeout -k 10 60 ./tools/sort_bench 28 5 | head -1 || exit $?
done
bash tools/sort_stamps.sh
