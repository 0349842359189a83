#!/bin/bash
# round-3: SpMV persistent form (tests + shapes), scan granule stride 32 vs
# 64 / 128, sort vector write-out A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_reduce.py tests/test_gpu_configs.py tests/test_gpu_scan.py -m gpu -q -x -k "spmv or gemv or csr or scan" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03f_tests.log 2>&1 || { tail -30 gpurun_out/r03f_tests.log; exit 1; }
tail -1 gpurun_out/r03f_tests.log
timeout -k 10 400 python -u tools/spmv_shapes.py > gpurun_out/r03f_spmv.txt 2>&1 || { cat gpurun_out/r03f_spmv.txt; exit 1; }
cat gpurun_out/r03f_spmv.txt
for i in 1 2 3; do
  for v in g32 g64 g128; do
    if [ $v = g32 ]; then unset DRHIP_LIB; else export DRHIP_LIB=$PWD/tools/var_r03/$v/libdrhip.so; fi
    timeout -k 10 120 python bench.py --no-cpu-baseline --only-ops c2_int32 --steps 30 > gpurun_out/r03f_ab.json 2>gpurun_out/r03f_ab.err || { tail gpurun_out/r03f_ab.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/r03f_ab.json')); o=d['ops']; print('$v', 'f32 scan', round(d['roofline']['launch_ms'],4), 'i32 scan', round(o['c2_int32']['scan_ms'],4), d['check']['ok'], o['c2_int32']['check']['ok'])"
  done
  for v in wo1 wo4; do
    if [ $v = wo1 ]; then unset DRHIP_LIB; else export DRHIP_LIB=$PWD/tools/var_r03/sort_wovec/libdrhip.so; fi
    timeout -k 10 120 python bench.py --no-cpu-baseline --only-ops sort --steps 20 > gpurun_out/r03f_sort.json 2>gpurun_out/r03f_sort.err || { tail gpurun_out/r03f_sort.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/r03f_sort.json')); o=d['ops']['sort']; print('$v', 'local sort', round(o['local_sort_ms'],4), o['check']['ok'])"
  done
done
