#!/bin/bash
# round-3: mhp suite on 1-4 MPI ranks, scan + sort + spmv tests, granule-
# stride A/B, sort pre-pass A/B (digit 1 counted in pass 0 vs the pre-pass),
# SpMV chunk shapes
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_cpp_shp.py -m gpu -k mhp -v --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r03e_mhp.log 2>&1 || { tail -40 gpurun_out/r03e_mhp.log; exit 1; }
grep -E "PASS|FAIL|SKIP" gpurun_out/r03e_mhp.log | tail -12
timeout -k 10 600 python -u -m pytest tests/test_gpu_scan.py tests/test_gpu_sort.py tests/test_gpu_reduce.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03e_tests.log 2>&1 || { tail -30 gpurun_out/r03e_tests.log; exit 1; }
tail -1 gpurun_out/r03e_tests.log
for i in 1 2 3; do
  for v in g16 g8 g32; do
    if [ $v = g16 ]; then unset DRHIP_LIB; else export DRHIP_LIB=$PWD/tools/var_r03/$v/libdrhip.so; fi
    timeout -k 10 120 python bench.py --no-cpu-baseline --only-ops c2_int32 --steps 30 > gpurun_out/r03e_ab.json 2>gpurun_out/r03e_ab.err || { tail gpurun_out/r03e_ab.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/r03e_ab.json')); o=d['ops']; print('$v', 'f32 scan', round(d['roofline']['launch_ms'],4), 'i32 scan', round(o['c2_int32']['scan_ms'],4), d['check']['ok'], o['c2_int32']['check']['ok'])"
  done
  for v in h0new h0old; do
    if [ $v = h0new ]; then unset DRHIP_LIB; else export DRHIP_LIB=$PWD/tools/var_r03/sort_h0cnt1/libdrhip.so; fi
    timeout -k 10 120 python bench.py --no-cpu-baseline --only-ops sort --steps 20 > gpurun_out/r03e_sort.json 2>gpurun_out/r03e_sort.err || { tail gpurun_out/r03e_sort.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/r03e_sort.json')); o=d['ops']['sort']; print('$v', 'local sort', round(o['local_sort_ms'],4), o['check']['ok'])"
  done
done
unset DRHIP_LIB
timeout -k 10 400 python -u tools/spmv_shapes.py > gpurun_out/r03e_spmv.txt 2>&1 || { cat gpurun_out/r03e_spmv.txt; exit 1; }
cat gpurun_out/r03e_spmv.txt
timeout -k 10 200 tools/gather_ceiling > gpurun_out/r03e_gather.txt 2>&1 || { cat gpurun_out/r03e_gather.txt; exit 1; }
cat gpurun_out/r03e_gather.txt
