#!/bin/bash
# round-3: mhp suite on 1-4 MPI ranks (one GPU), scan tests at the new
# granule stride, granule-stride A/B (8 / 16 default / 32 / 64 B per tile)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_cpp_shp.py -m gpu -k mhp -v --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r03d_mhp.log 2>&1 || { tail -40 gpurun_out/r03d_mhp.log; exit 1; }
grep -E "PASS|FAIL|SKIP" gpurun_out/r03d_mhp.log | tail -12
timeout -k 10 600 python -u -m pytest tests/test_gpu_scan.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03d_scan.log 2>&1 || { tail -30 gpurun_out/r03d_scan.log; exit 1; }
tail -1 gpurun_out/r03d_scan.log
for i in 1 2 3; do
  for v in g16 g8 g32 g64; do
    if [ $v = g16 ]; then unset DRHIP_LIB; else export DRHIP_LIB=$PWD/tools/var_r03/$v/libdrhip.so; fi
    timeout -k 10 120 python bench.py --no-cpu-baseline --only-ops c2_int32 --steps 30 > gpurun_out/r03d_ab.json 2>gpurun_out/r03d_ab.err || { tail gpurun_out/r03d_ab.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/r03d_ab.json')); o=d['ops']; print('$v', 'f32 scan', round(d['roofline']['launch_ms'],4), 'i32 scan', round(o['c2_int32']['scan_ms'],4), d['check']['ok'], o['c2_int32']['check']['ok'])"
  done
done
