#!/bin/bash
# round 6, pass q: (1) the banded SpMV's LDS x window for 8-byte indices
# (DRHIP_SPMV_I64_WIN=1, at 8 and 6 waves/SIMD) vs global gathers (default):
# parity, then interleaved bench runs of the int64 gemv ops; (2) the pool
# reproducer with copy and kernel fills (tools/r06/gpu_p.sh).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06q
mkdir -p $O
for v in i64w8 i64w6; do
  DRHIP_LIB=$PWD/tools/var6/$v/libdrhip.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 \
    --timeout-method thread tests/test_gpu_elementwise.py -k spmv -m gpu > $O/${v}_pytest.txt 2>&1; rc=$?
  echo "$v parity rc $rc: $(tail -1 $O/${v}_pytest.txt)"
  [ $rc -ne 0 ] && exit $rc
done
for rep in 1 2 3; do
  for v in base i64w8 i64w6; do
    if [ $v = base ]; then L=$PWD/distributed-ranges_amd/libdrhip.so; else L=$PWD/tools/var6/$v/libdrhip.so; fi
    DRHIP_LIB=$L timeout -k 10 300 python3 bench.py --only-ops gemv_banded,gemv_banded_i64,gemv_i64 --log2n 24 --steps 10 \
      --warmup 2 --no-cpu-baseline > $O/bench_${v}_$rep.json 2> $O/bench_${v}_$rep.err; rc=$?
    [ $rc -ne 0 ] && { tail -5 $O/bench_${v}_$rep.err; exit $rc; }
    python3 -c "
import json; o=json.load(open('$O/bench_${v}_$rep.json'))['ops']
print('rep $rep %-6s banded %.4f (%.3f)  banded_i64 %.4f (%.3f)  random_i64 %.3f  ok %s' % ('$v', o['gemv_banded']['kernel_ms'], o['gemv_banded']['frac'], o['gemv_banded_i64']['kernel_ms'], o['gemv_banded_i64']['frac'], o['gemv_i64']['kernel_ms'], all(o[k]['check']['ok'] for k in o)))"
  done
done
bash tools/r06/gpu_p.sh
