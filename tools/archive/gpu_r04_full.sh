#!/bin/bash
# round-4 evidence at HEAD: the whole -m gpu suite, smoke(), the default
# bench line, rocprofv3 kernel stats of the full bench (every op), the
# FETCH_SIZE / WRITE_SIZE PMC passes of the headline, and the scan U A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04_pytest_gpu.log 2>&1; rc=$?
tail -4 gpurun_out/r04_pytest_gpu.log; [ $rc -eq 0 ] || { grep -B2 -A40 "FAILED\|Error" gpurun_out/r04_pytest_gpu.log | head -80; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1
timeout -k 10 600 python -u bench.py > gpurun_out/r04_bench_n1.json 2> gpurun_out/r04_bench_n1.err || { tail -20 gpurun_out/r04_bench_n1.err; exit 1; }
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/r04_bench_n1.json"))
print('value', d['value'], 'ms', d['ms_per_step'], 'frac', d['roofline']['frac'], 'check', d['check']['ok'])
for k, v in d['ops'].items():
    print(k, {kk: (round(vv, 4) if isinstance(vv, float) else vv) for kk, vv in v.items()
              if kk in ('ms', 'kernel_ms', 'frac', 'local_sort_ms', 'reduce_frac', 'scan_frac', 'graph_ms',
                        'predicted_speedup_8')}, v.get('check', {}).get('ok') if isinstance(v.get('check'), dict) else '')
PY
rm -rf gpurun_out/prof_r04
timeout -s KILL 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_r04" -o prof --output-format csv \
  -- python3 "$R/bench.py" --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/prof_r04.log 2>&1 || { tail -20 gpurun_out/prof_r04.log; exit 1; }
f=$(find gpurun_out/prof_r04 -name "*kernel_stats.csv" | head -1)
cp "$f" gpurun_out/r04_kernel_stats_bench.csv
head -30 gpurun_out/r04_kernel_stats_bench.csv | cut -c1-180
BENCH_ARGS="--no-ops" bash tools/pmc.sh || exit 1
timeout -k 10 300 python -u tools/reduce_ab.py u32=default u16=tools/abvar/scan_u16/libdrhip.so | tee gpurun_out/r04_scan_u16_ab.txt
