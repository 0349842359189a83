#!/bin/bash
# round 6, pass d: the row-window SpMV (drhip_spmv_csr_window) -- parity
# tests, C4 through shp::gemv, and bench A/B against drhip_spmv_csr in
# interleaved runs on one box; the new allocator tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06d
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_elementwise.py -k spmv tests/test_gpu_memory.py > $O/pytest.txt 2>&1; rc=$?
echo "pytest rc $rc: $(tail -2 $O/pytest.txt | tr '\n' ' ')"
[ $rc -ne 0 ] && exit $rc
for k in banded random; do
  timeout -k 10 400 tests/cpp/bin/config_tests c4 26 8 --kind $k --index i64 > $O/c4_$k.txt 2>&1; rc=$?
  echo "c4 $k rc $rc: $(grep '^{' $O/c4_$k.txt | cut -c1-400)"
  [ $rc -ne 0 ] && exit $rc
done
OPS=gemv_banded,gemv,gemv_banded_i64,gemv_i64
for rep in 1 2 3; do
  for v in window plain; do
    if [ $v = plain ]; then export DRHIP_BENCH_SPMV_PLAIN=1; else unset DRHIP_BENCH_SPMV_PLAIN; fi
    timeout -k 10 300 python3 bench.py --only-ops $OPS --log2n 24 --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_${v}_$rep.json 2> $O/bench_${v}_$rep.err; rc=$?
    [ $rc -ne 0 ] && { tail -5 $O/bench_${v}_$rep.err; exit $rc; }
    python3 -c "
import json; d=json.load(open('$O/bench_${v}_$rep.json'))['ops']
print('rep $rep $v', {k: (round(d[k]['kernel_ms'], 4), round(d[k]['frac'], 3), d[k]['check']['ok']) for k in '$OPS'.split(',')})"
  done
done
