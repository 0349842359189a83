#!/bin/bash
# round-3: template (user-operator) look-back scan at 32 slots per thread
# (chunked piece scan) vs the shipped 16: C++ suite on the variant, then
# dense_bench A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 tools/var_r03/lb32/shp_tests > gpurun_out/r03k_shp_lb32.log 2>&1 || { tail -30 gpurun_out/r03k_shp_lb32.log; exit 1; }
tail -2 gpurun_out/r03k_shp_lb32.log
timeout -k 10 300 tools/var_r03/lb32/shp_tests --devicesCount 3 > gpurun_out/r03k_shp3_lb32.log 2>&1 || { tail -30 gpurun_out/r03k_shp3_lb32.log; exit 1; }
tail -2 gpurun_out/r03k_shp3_lb32.log
for i in 1 2 3; do
  for v in base lb32; do
    if [ $v = base ]; then exe=tests/cpp/bin/dense_bench; else exe=tools/var_r03/lb32/dense_bench; fi
    timeout -k 10 120 $exe > gpurun_out/r03k_dense.txt 2>&1 || { cat gpurun_out/r03k_dense.txt; exit 1; }
    python3 -c "
import json
for l in open('gpurun_out/r03k_dense.txt'):
    if l.startswith('{'):
        d=json.loads(l)
        if d.get('op') in ('scan_lambda_op',):
            print('$v', d['op'], d.get('ms'), d.get('frac'), d.get('check'))
"
  done
done
