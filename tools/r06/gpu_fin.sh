#!/bin/bash
# round 6, final pass: evidence at HEAD -- the whole -m gpu suite, smoke, the
# default bench line, its rocprofv3 kernel stats, and the N = 2 / N = 4
# rehearsals of the multi-rank bench path on one GPU (gloo, small sizes).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06fin
mkdir -p $O
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q -rs --timeout 600 --timeout-method thread > $O/pytest_gpu.txt 2>&1; rc=$?
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
print('value %.4g ms %.4f frac %.4f traffic %s' % (d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['traffic']))
print('cpu_baseline', {k: d['cpu_baseline'].get(k) for k in ('value', 'unit', 'cores', 'kind')})
for k, v in d.get('ops', {}).items():
    ms = v.get('kernel_ms', v.get('local_sort_ms', v.get('ms')))
    print(' ', k, None if ms is None else round(ms, 4), round(v.get('frac', 0), 3), v.get('check', {}).get('ok') if isinstance(v.get('check'), dict) else '')"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o bench --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/prof.log 2>&1; rc=$?
echo "rocprof rc $rc"
[ $rc -ne 0 ] && exit $rc
for np in 2 4; do
  NPROC=$np bash tools/bench_2rank_1gpu.sh > $O/rehearsal_n$np.json 2> $O/rehearsal_n$np.err; rc=$?
  echo "rehearsal N=$np rc $rc"
  [ $rc -ne 0 ] && { tail -20 $O/rehearsal_n$np.err; exit $rc; }
  python3 -c "
import json; d=[json.loads(l) for l in open('$O/rehearsal_n$np.json') if l.startswith('{')][-1]
bad = [k for k, v in d.get('ops', {}).items() if isinstance(v, dict) and isinstance(v.get('check'), dict) and not v['check'].get('ok')]
print('  N=$np n_gpus', d['n_gpus'], 'check', d['check']['ok'], 'ops failing', bad)"
done
