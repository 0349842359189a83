#!/bin/bash
# round-3: scan granule A/B on one box (P62 8-B word vs the round-2 16-B sc1
# granule build in tools/var_r03/scan_g16), SpMV bench-vs-sweep gap, chunk shapes
set -o pipefail
mkdir -p gpurun_out
for i in 1 2 3; do
  for v in new old; do
    if [ $v = old ]; then export DRHIP_LIB=$PWD/tools/var_r03/scan_g16/libdrhip.so; else unset DRHIP_LIB; fi
    timeout -k 10 120 python bench.py --no-cpu-baseline --only-ops c2_int32 --steps 30 > gpurun_out/r03c_ab.json 2>gpurun_out/r03c_ab.err || { tail gpurun_out/r03c_ab.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/r03c_ab.json')); o=d['ops']; print('$v', 'f32 scan', round(d['roofline']['launch_ms'],4), 'reduce', round(o['reduce']['ms'],4), 'i32 scan', round(o['c2_int32']['scan_ms'],4), d['check']['ok'], o['c2_int32']['check']['ok'])"
  done
done
unset DRHIP_LIB
timeout -k 10 300 python -u tools/spmv_gap.py > gpurun_out/r03c_spmv_gap.txt 2>&1 || { cat gpurun_out/r03c_spmv_gap.txt; exit 1; }
cat gpurun_out/r03c_spmv_gap.txt
timeout -k 10 300 python -u tools/spmv_npb.py > gpurun_out/r03c_spmv_npb.txt 2>&1 || { cat gpurun_out/r03c_spmv_npb.txt; exit 1; }
cat gpurun_out/r03c_spmv_npb.txt
