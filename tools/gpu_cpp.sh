#!/bin/bash
# C++ drop-in suite + the template-kernel bench (dense_bench), one GPU.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_cpp_shp.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/cpp.log 2>&1
rc=$?; grep -E "FAILED|passed|failed|exception" gpurun_out/cpp.log | tail -30
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 tests/cpp/bin/dense_bench 15 15 10 > gpurun_out/dense_bench.log 2>&1
rc=$?; cat gpurun_out/dense_bench.log; exit $rc
