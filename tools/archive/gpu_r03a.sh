#!/bin/bash
# round-3 check: the fixed nxcd paths, the config-size tests with output, one bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_sort.py -q -k "nxcd or concurrent" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03a_sort.log 2>&1 || { tail -20 gpurun_out/r03a_sort.log; exit 1; }
tail -2 gpurun_out/r03a_sort.log
timeout -k 10 300 tests/cpp/bin/config_tests 31 8 --threads 16 > gpurun_out/r03a_c3.json 2>&1 || { cat gpurun_out/r03a_c3.json; exit 1; }
cat gpurun_out/r03a_c3.json
timeout -k 10 400 python -u bench.py > gpurun_out/r03a_bench.json 2> gpurun_out/r03a_bench.err || { tail -20 gpurun_out/r03a_bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r03a_bench.json'))
print('value', d['value'], 'ms', d['ms_per_step'], 'frac', d['roofline']['frac'])
for k,v in d['ops'].items():
    print(k, {kk: vv for kk, vv in v.items() if kk in ('ms','kernel_ms','frac','local_sort_ms','input_copy_ms','reduce_frac','scan_frac','ok')}, v.get('check',{}).get('ok'))
"
