#!/bin/bash
# round 6, pass l: random C4 SpMV with nontemporal colind/vals loads
# (DRHIP_SPMV_NT=1: the 5.4 GB stream marked streaming, so that x -- 256 MB,
# the Infinity Cache's size -- might stay cached for the gathers) vs the
# default cached loads; banded alongside.  Parity, then interleaved bench runs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06l
mkdir -p $O
DRHIP_LIB=$PWD/tools/var6/spmvnt/libdrhip.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 \
  --timeout-method thread tests/test_gpu_elementwise.py -k spmv -m gpu > $O/spmvnt_pytest.txt 2>&1; rc=$?
echo "spmvnt parity rc $rc: $(tail -1 $O/spmvnt_pytest.txt)"
[ $rc -ne 0 ] && exit $rc
for rep in 1 2 3; do
  for v in base spmvnt; do
    if [ $v = base ]; then L=$PWD/distributed-ranges_amd/libdrhip.so; else L=$PWD/tools/var6/$v/libdrhip.so; fi
    DRHIP_LIB=$L timeout -k 10 300 python3 bench.py --only-ops gemv_banded,gemv --log2n 24 --steps 10 --warmup 2 \
      --no-cpu-baseline > $O/bench_${v}_$rep.json 2> $O/bench_${v}_$rep.err; rc=$?
    [ $rc -ne 0 ] && { tail -5 $O/bench_${v}_$rep.err; exit $rc; }
    python3 -c "
import json; o=json.load(open('$O/bench_${v}_$rep.json'))['ops']
print('rep $rep %-7s banded %.4f ms  random %.3f ms  ok %s %s' % ('$v', o['gemv_banded']['kernel_ms'], o['gemv']['kernel_ms'], o['gemv_banded']['check']['ok'], o['gemv']['check']['ok']))"
  done
done
