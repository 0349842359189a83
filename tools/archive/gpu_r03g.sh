#!/bin/bash
# round-3: scan granule stride 128 (default) vs 256 / 512, template scan at a
# 128-B granule stride (C++ suite + dense_bench), SpMV/scan tests, full bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_scan.py tests/test_cpp_shp.py tests/test_gpu_configs.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03g_tests.log 2>&1 || { tail -30 gpurun_out/r03g_tests.log; exit 1; }
tail -1 gpurun_out/r03g_tests.log
for i in 1 2 3; do
  for v in g128 g256 g512; do
    if [ $v = g128 ]; then unset DRHIP_LIB; else export DRHIP_LIB=$PWD/tools/var_r03/$v/libdrhip.so; fi
    timeout -k 10 120 python bench.py --no-cpu-baseline --only-ops c2_int32 --steps 30 > gpurun_out/r03g_ab.json 2>gpurun_out/r03g_ab.err || { tail gpurun_out/r03g_ab.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/r03g_ab.json')); o=d['ops']; print('$v', 'f32 scan', round(d['roofline']['launch_ms'],4), 'i32 scan', round(o['c2_int32']['scan_ms'],4), d['check']['ok'], o['c2_int32']['check']['ok'])"
  done
done
unset DRHIP_LIB
timeout -k 10 400 python -u bench.py --steps 20 --warmup 3 > gpurun_out/r03g_bench.json 2> gpurun_out/r03g_bench.err || { tail -20 gpurun_out/r03g_bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r03g_bench.json'))
print('value', d['value'], 'ms', d['ms_per_step'], 'frac', d['roofline']['frac'])
for k,v in d['ops'].items():
    print(k, {kk: (round(vv,4) if isinstance(vv,float) else vv) for kk, vv in v.items() if kk in ('ms','kernel_ms','frac','local_sort_ms','reduce_frac','scan_frac')})
"
