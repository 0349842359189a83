#!/bin/bash
# sort parity + timing + per-kernel profile + stamps
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_sort.py -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/pytest_sort.log 2>&1
rc=$?; tail -n 2 gpurun_out/pytest_sort.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 60 ./tools/sort_bench 28 5 || exit $?
rm -rf gpurun_out/sortprof
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/sortprof" -o run --output-format csv \
  -- ./tools/sort_bench 28 3 > gpurun_out/sortprof.log 2>&1 || exit $?
VARIANTS="stamps stamps0" bash tools/sort_stamps.sh
