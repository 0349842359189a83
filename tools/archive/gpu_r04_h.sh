#!/bin/bash
# round 4: C++ blocking-call overhead by sync mode; sort parity at default NT=256
set -o pipefail
mkdir -p gpurun_out
for m in spin auto yield spin; do
  DRHIP_SYNC=$m timeout -k 10 120 ./tests/cpp/bin/shp_bench --overhead 0 | grep '^{' | tee -a gpurun_out/r04h_overhead.txt || exit 1
done
bash tools/sort_parity.sh
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_cpp_shp.py -k "shp_suite or config" > gpurun_out/r04h_cpp.log 2>&1; rc=$?; tail -3 gpurun_out/r04h_cpp.log; [ $rc -eq 0 ] || exit 1
GATHER_PANELS=1 timeout -k 10 180 ./tools/gather_ceiling | tee gpurun_out/r04h_gather_panels.txt
timeout -k 10 300 python -u tools/reduce_ab.py u32=default u16=tools/abvar/scan_u16/libdrhip.so | tee gpurun_out/r04h_scan_u16_ab.txt
