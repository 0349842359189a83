#!/bin/bash
# round-3: nonzero-split SpMV -- parity (irregular rows both paths, the
# parity matrix set and C4 with DRHIP_SPMV_SPLIT=1), then shapes A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_elementwise.py -m gpu -q -x -k "spmv" --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r03m_t1.log 2>&1 || { tail -30 gpurun_out/r03m_t1.log; exit 1; }
tail -1 gpurun_out/r03m_t1.log
DRHIP_SPMV_SPLIT=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_elementwise.py tests/test_gpu_configs.py -m gpu -q -x -k "spmv or c4" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03m_t2.log 2>&1 || { tail -30 gpurun_out/r03m_t2.log; exit 1; }
tail -1 gpurun_out/r03m_t2.log
timeout -k 10 400 python -u tools/spmv_shapes.py > gpurun_out/r03m_spmv.txt 2>&1 || { cat gpurun_out/r03m_spmv.txt; exit 1; }
cat gpurun_out/r03m_spmv.txt
