#!/bin/bash
# round-3 evidence at HEAD: the whole -m gpu suite, smoke(), the default bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/r03_pytest_gpu.txt 2>&1
rc=$?; tail -3 gpurun_out/r03_pytest_gpu.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_smoke.txt 2>&1 || { cat gpurun_out/r03_smoke.txt; exit 1; }
cat gpurun_out/r03_smoke.txt
timeout -k 10 400 python -u bench.py > gpurun_out/r03_bench_default.json 2> gpurun_out/r03_bench_default.err || { tail -20 gpurun_out/r03_bench_default.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r03_bench_default.json'))
print('value', d['value'], 'ms', d['ms_per_step'], 'frac', d['roofline']['frac'], 'check', d['check']['ok'])
for k,v in d['ops'].items():
    print(k, {kk: (round(vv,4) if isinstance(vv,float) else vv) for kk, vv in v.items() if kk in ('ms','kernel_ms','frac','local_sort_ms','reduce_frac','scan_frac')}, v.get('check',{}).get('ok') if isinstance(v.get('check'),dict) else v.get('check'))
"
