#!/bin/bash
# round-3: x-window threshold test, all SpMV/stencil tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_elementwise.py -m gpu -q -x -k "spmv or stencil" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03t.log 2>&1 || { tail -30 gpurun_out/r03t.log; exit 1; }
tail -1 gpurun_out/r03t.log
