#!/bin/bash
# round 6, pass e: evidence at HEAD -- the whole -m gpu suite, smoke, the
# default bench line, and the rocprofv3 kernel stats of the same bench.
# Each GPU step under its own time limit; stop at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06e
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q -rs --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1; rc=$?
echo "pytest rc $rc: $(tail -1 $O/pytest_gpu.txt)"
[ $rc -ne 0 ] && { grep -E "FAILED|Error" $O/pytest_gpu.txt | tail -20; exit $rc; }
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1; rc=$?
echo "smoke rc $rc: $(tail -1 $O/smoke.txt)"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err; rc=$?
echo "bench rc $rc"
[ $rc -ne 0 ] && { tail -20 $O/bench.err; exit $rc; }
python3 -c "
import json; d=json.load(open('$O/bench.json'))
print('value', d['value'], 'ms', d['ms_per_step'], 'frac', d['roofline']['frac'])
for k, v in d.get('ops', {}).items():
    print(' ', k, round(v.get('kernel_ms', v.get('ms', 0)), 4), round(v.get('frac', 0), 3), v.get('check', {}).get('ok'))"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o bench --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/prof.log 2>&1; rc=$?
echo "rocprof rc $rc"
exit $rc
