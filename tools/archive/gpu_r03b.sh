#!/bin/bash
# round-3: scan granule change (tests + A/B vs the 16-B sc1 granule build), SpMV bench gap
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_scan.py -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03b_tests.log 2>&1 || { tail -30 gpurun_out/r03b_tests.log; exit 1; }
tail -2 gpurun_out/r03b_tests.log
for i in 1 2 3; do
  for v in new old; do
    if [ $v = old ]; then export DRHIP_LIB=$PWD/tools/var_r03/scan_g16/libdrhip.so; else unset DRHIP_LIB; fi
    timeout -k 10 120 python bench.py --no-ops --no-cpu-baseline --steps 30 > gpurun_out/r03b_ab.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/r03b_ab.json')); print('$v', round(d['roofline']['launch_ms'],4), round(d['ops']['reduce']['ms'],4), d['check']['ok'])"
  done
done
unset DRHIP_LIB
timeout -k 10 300 python -u tools/spmv_npb.py > gpurun_out/r03b_spmv_npb.txt 2>&1 || { cat gpurun_out/r03b_spmv_npb.txt; exit 1; }
cat gpurun_out/r03b_spmv_npb.txt
