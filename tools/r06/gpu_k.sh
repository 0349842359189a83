#!/bin/bash
# round 6, pass k: the C2 step's scan taking the reduce blocks' TAIL tiles
# first (DRHIP_WAVE_GIVEN_ORDER=1: what the step's reduce read last), with nt
# loads (order1) and cached loads (order1c), vs the start-order default:
# scan parity with each variant, then interleaved headline-only bench runs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06k
mkdir -p $O
for v in order1 order1c; do
  DRHIP_LIB=$PWD/tools/var6/$v/libdrhip.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 \
    --timeout-method thread tests/test_gpu_scan.py tests/test_gpu_configs.py -k "scan or c2" -m gpu > $O/${v}_pytest.txt 2>&1; rc=$?
  echo "$v parity rc $rc: $(tail -1 $O/${v}_pytest.txt)"
  [ $rc -ne 0 ] && { grep -E "FAILED|Error" $O/${v}_pytest.txt | tail -10; exit $rc; }
done
for rep in 1 2 3; do
  for v in base order1 order1c; do
    if [ $v = base ]; then L=$PWD/distributed-ranges_amd/libdrhip.so; else L=$PWD/tools/var6/$v/libdrhip.so; fi
    DRHIP_LIB=$L timeout -k 10 300 python3 bench.py --no-ops --steps 20 --warmup 5 --no-cpu-baseline \
      > $O/bench_${v}_$rep.json 2> $O/bench_${v}_$rep.err; rc=$?
    [ $rc -ne 0 ] && { tail -5 $O/bench_${v}_$rep.err; exit $rc; }
    python3 -c "
import json; d=json.load(open('$O/bench_${v}_$rep.json')); o=d['ops']
print('rep $rep %-8s step %.4f ms  reduce %.4f  scan %.4f  check %s' % ('$v', d['ms_per_step'], o['reduce']['ms'], o['inclusive_scan']['ms'], d['check']['ok']))"
  done
done
