#!/bin/bash
# round-3: staged two-span reduce for transform(zip(a, b)) -- C++ suite, then
# dense_bench ops
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_cpp_shp.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03s_t.log 2>&1 || { tail -30 gpurun_out/r03s_t.log; exit 1; }
tail -1 gpurun_out/r03s_t.log
for i in 1 2 3; do
  timeout -k 10 120 tests/cpp/bin/dense_bench > gpurun_out/r03s_dense.txt 2>&1 || { cat gpurun_out/r03s_dense.txt; exit 1; }
  grep -E "reduce_zip_transform|reduce_lambda_op|zip_for_each|enumerate_for_each" gpurun_out/r03s_dense.txt
done
