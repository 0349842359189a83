#!/bin/bash
# round-3: SpMV x window follow-up: default (XW 2048, 8 waves) vs 7 waves
# (w7, no spills), XW 1024, no window (xw0); parity on the default first;
# then the bench's own gemv ops
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_elementwise.py tests/test_gpu_configs.py tests/test_cpp_shp.py -m gpu -q -x -k "spmv or c4 or gemv or sparse or suite" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03o_t.log 2>&1 || { tail -30 gpurun_out/r03o_t.log; exit 1; }
tail -1 gpurun_out/r03o_t.log
for i in 1 2; do
  for v in xw2048 w7 xw1024 xw0; do
    if [ $v = xw2048 ]; then unset DRHIP_LIB; else export DRHIP_LIB=$PWD/tools/var_r03/$v/libdrhip.so; fi
    timeout -k 10 200 python -u tools/spmv_shapes.py default > gpurun_out/r03o_spmv.txt 2>&1 || { cat gpurun_out/r03o_spmv.txt; exit 1; }
    grep -v amdgpu.ids gpurun_out/r03o_spmv.txt | sed "s/^/$v /"
  done
done
unset DRHIP_LIB
timeout -k 10 200 python bench.py --no-cpu-baseline --only-ops gemv_banded,gemv_random --steps 20 > gpurun_out/r03o_bench.json 2>gpurun_out/r03o_bench.err || { tail gpurun_out/r03o_bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r03o_bench.json'))
for k,v in d['ops'].items(): print(k, round(v['kernel_ms'],4), round(v['frac'],4), v['check']['ok'])"
