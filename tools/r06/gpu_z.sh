#!/bin/bash
# round 6, pass z: the few-digit ranking gated by the pass histogram (fk4), + the pre-pass probe (fk4h), vs base
# for the <= K digits of a wave's first round: few4 K = 4, few2 K = 2) vs u2
# (uniform fast paths only): parity, skew probe, bench sort op, interleaved.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06z
mkdir -p $O
for v in fk4 fk4h; do
  DRHIP_LIB=$PWD/tools/var6/$v/libdrhip.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 \
    --timeout-method thread tests/test_gpu_sort.py -m gpu > $O/${v}_pytest.txt 2>&1; rc=$?
  echo "$v parity rc $rc: $(tail -1 $O/${v}_pytest.txt)"
  [ $rc -ne 0 ] && { grep -E "FAILED|Error" $O/${v}_pytest.txt | tail -10; exit $rc; }
done
for rep in 1 2 3; do
  for v in base fk4 fk4h; do
    L=$PWD/tools/var6/$v/libdrhip.so; [ $v = base ] && L=$PWD/distributed-ranges_amd/libdrhip.so; DRHIP_LIB=$L timeout -k 10 300 python3 bench.py --only-ops sort --log2n 24 --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_${v}_$rep.json 2>/dev/null || exit 1
    python3 -c "
import json; o=json.load(open('$O/bench_${v}_$rep.json'))['ops']['sort']; print('rep $rep %-4s bench sort local %.4f ms ok %s' % ('$v', o['local_sort_ms'], o['check']['ok']))"
  done
done
for v in base fk4 fk4h; do
  L=$PWD/tools/var6/$v/libdrhip.so; [ $v = base ] && L=$PWD/distributed-ranges_amd/libdrhip.so; echo "== $v"; DRHIP_LIB=$L timeout -k 10 300 python3 tools/r06/sort_skew_probe.py 2>&1 | grep -v amdgpu.ids | tee $O/skew_$v.txt || exit 1
done
