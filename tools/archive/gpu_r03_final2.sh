#!/bin/bash
# round-3 evidence at HEAD: the whole -m gpu suite, smoke(), the default
# bench line, rocprofv3 kernel stats of the bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/r03_pytest_gpu.txt 2>&1
rc=$?; tail -3 gpurun_out/r03_pytest_gpu.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_smoke.txt 2>&1 || { cat gpurun_out/r03_smoke.txt; exit 1; }
tail -1 gpurun_out/r03_smoke.txt
timeout -k 10 400 python -u bench.py > gpurun_out/r03_bench_default.json 2> gpurun_out/r03_bench_default.err || { tail -20 gpurun_out/r03_bench_default.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r03_bench_default.json'))
print('value', d['value'], 'ms', d['ms_per_step'], 'frac', d['roofline']['frac'], 'check', d['check']['ok'])
for k,v in d['ops'].items():
    print(k, {kk: (round(vv,4) if isinstance(vv,float) else vv) for kk, vv in v.items() if kk in ('ms','kernel_ms','frac','local_sort_ms','reduce_frac','scan_frac')})
"
rm -rf gpurun_out/prof_r03b
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_r03b" -o prof --output-format csv \
  -- python3 "$R/bench.py" --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/prof_r03b.log 2>&1 || { tail -20 gpurun_out/prof_r03b.log; exit 1; }
f=$(find gpurun_out/prof_r03b -name "*kernel_stats.csv" | head -1)
cp "$f" gpurun_out/r03b_kernel_stats_bench.csv
grep "^{" gpurun_out/prof_r03b.log | tail -1 > gpurun_out/r03b_bench_under_rocprof.json
echo done
