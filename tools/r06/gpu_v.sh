#!/bin/bash
# round 6, pass v: the sort's skew fast paths with early-exit checks (u2) vs
# the round-5 sort (r5: no fast paths, passes count the next digit) and u1h:
# parity for u2, then interleaved bench sort ops and skew probes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06v
mkdir -p $O
DRHIP_LIB=$PWD/tools/var6/u2/libdrhip.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 \
  --timeout-method thread tests/test_gpu_sort.py -m gpu > $O/u2_pytest.txt 2>&1; rc=$?
echo "u2 parity rc $rc: $(tail -1 $O/u2_pytest.txt)"
[ $rc -ne 0 ] && exit $rc
for rep in 1 2 3; do
  for v in r5 u1h u2; do
    L=$PWD/tools/var6/$v/libdrhip.so
    DRHIP_LIB=$L timeout -k 10 300 python3 bench.py --only-ops sort --log2n 24 --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_${v}_$rep.json 2>/dev/null || exit 1
    python3 -c "
import json; o=json.load(open('$O/bench_${v}_$rep.json'))['ops']['sort']; print('rep $rep %-4s bench sort local %.4f ms ok %s' % ('$v', o['local_sort_ms'], o['check']['ok']))"
  done
done
for v in r5 u1h u2; do
  echo "== $v"; DRHIP_LIB=$PWD/tools/var6/$v/libdrhip.so timeout -k 10 300 python3 tools/r06/sort_skew_probe.py 2>&1 | grep -v amdgpu.ids | tee $O/skew_$v.txt || exit 1
done
