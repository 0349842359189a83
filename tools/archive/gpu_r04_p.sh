#!/bin/bash
# round 4: sort pass 0 as a one-shot grid (no claims) vs the persistent claim loop, 2^28 u32, 3 interleaved rounds,
# rocprof per-pass times of each
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/r04p_sort_ab.txt
for r in 1 2 3; do
  for v in default p0oneshot; do
    if [ $v = default ]; then unset DRHIP_LIB; else export DRHIP_LIB=$R/tools/abvar/$v/libdrhip.so; fi
    timeout -k 10 120 python -u bench.py --only-ops sort --no-cpu-baseline > /tmp/s.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.loads(open('/tmp/s.json').read().strip().splitlines()[-1]);s=d['ops']['sort'];print('$r $v', round(s['local_sort_ms'],4), s['check']['ok'])" | tee -a gpurun_out/r04p_sort_ab.txt
  done
done
unset DRHIP_LIB
for v in default p0oneshot; do
  if [ $v != default ]; then export DRHIP_LIB=$R/tools/abvar/$v/libdrhip.so; fi
  rm -rf gpurun_out/prof_p_$v
  timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_p_$v" -o prof --output-format csv -- python3 "$R/bench.py" --only-ops sort --no-cpu-baseline > /dev/null 2>&1 || exit 1
  f=$(find gpurun_out/prof_p_$v -name "*kernel_stats.csv" | head -1)
  echo "== $v" | tee -a gpurun_out/r04p_sort_ab.txt
  python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    if 'radix' in r['Name']: print('  ', r['Name'][:70], r['Calls'], round(float(r['AverageNs'])/1e3,1))
" | tee -a gpurun_out/r04p_sort_ab.txt
done
