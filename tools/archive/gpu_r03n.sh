#!/bin/bash
# round-3: LDS-cached x window in the CSR-stream SpMV (XW = 2048 default,
# occupancy 5) vs no window (xw0), the window at 8 waves/SIMD (xw_w8), a
# 512-entry window (xw512); SpMV parity on the default build first
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_elementwise.py tests/test_gpu_configs.py -m gpu -q -x -k "spmv or c4" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03n_t.log 2>&1 || { tail -30 gpurun_out/r03n_t.log; exit 1; }
tail -1 gpurun_out/r03n_t.log
for i in 1 2; do
  for v in xw2048 xw0 xw_w8 xw512; do
    if [ $v = xw2048 ]; then unset DRHIP_LIB; else export DRHIP_LIB=$PWD/tools/var_r03/$v/libdrhip.so; fi
    timeout -k 10 200 python -u tools/spmv_shapes.py default > gpurun_out/r03n_spmv.txt 2>&1 || { cat gpurun_out/r03n_spmv.txt; exit 1; }
    grep -v amdgpu.ids gpurun_out/r03n_spmv.txt | sed "s/^/$v /"
  done
done
