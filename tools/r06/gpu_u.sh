#!/bin/bash
# round 6, pass u: the shipped sort (wave-uniform fast paths, every position
# counted in the pre-pass): sort parity incl. the skewed-digit tests, the C3
# config tests, the skew probe and the bench's sort op.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06u
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_sort.py \
  tests/test_gpu_configs.py -k "sort or c3" -m gpu > $O/pytest.txt 2>&1; rc=$?
echo "parity rc $rc: $(tail -1 $O/pytest.txt)"
[ $rc -ne 0 ] && { grep -E "FAILED|Error" $O/pytest.txt | tail -10; exit $rc; }
timeout -k 10 300 python3 tools/r06/sort_skew_probe.py 2>&1 | grep -v amdgpu.ids | tee $O/skew.txt || exit 1
for rep in 1 2; do
  timeout -k 10 300 python3 bench.py --only-ops sort --log2n 24 --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_$rep.json 2>/dev/null || exit 1
  python3 -c "
import json; o=json.load(open('$O/bench_$rep.json'))['ops']['sort']; print('bench sort local %.4f ms frac %.3f ok %s' % (o['local_sort_ms'], o['frac'], o['check']['ok']))"
done
