#!/bin/bash
# sort parity (every -m gpu sort test incl. the C3 config) + timing
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_sort.py tests/test_gpu_configs.py -m gpu -q -x --timeout 200 --timeout-method thread -k "sort or c3" > gpurun_out/pytest_sort.log 2>&1
rc=$?; tail -n 3 gpurun_out/pytest_sort.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 60 ./tools/sort_bench 28 5 && timeout -k 10 60 ./tools/sort_bench 26 5
