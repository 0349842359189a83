#!/bin/bash
# round 6, pass ab: 512-thread SpMV blocks (DRHIP_SPMV_BLOCK=512, 4096-slot
# chunks: twice the rows and bytes per block, the same per thread) vs the
# shipped 256-thread blocks: parity, then interleaved bench runs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06ab
mkdir -p $O
DRHIP_LIB=$PWD/tools/var6/b512/libdrhip.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 \
  --timeout-method thread tests/test_gpu_elementwise.py tests/test_gpu_configs.py -k "spmv or gemv_row_tile" -m gpu > $O/b512_pytest.txt 2>&1; rc=$?
echo "b512 parity rc $rc: $(tail -1 $O/b512_pytest.txt)"
[ $rc -ne 0 ] && { grep -E "FAILED|Error" $O/b512_pytest.txt | tail; exit $rc; }
for rep in 1 2 3; do
  for v in base b512; do
    L=$PWD/tools/var6/$v/libdrhip.so; [ $v = base ] && L=$PWD/distributed-ranges_amd/libdrhip.so
    DRHIP_LIB=$L timeout -k 10 300 python3 bench.py --only-ops gemv_banded,gemv,gemv_banded_i64 --log2n 24 --steps 10 \
      --warmup 2 --no-cpu-baseline > $O/bench_${v}_$rep.json 2>/dev/null || exit 1
    python3 -c "
import json; o=json.load(open('$O/bench_${v}_$rep.json'))['ops']
print('rep $rep %-5s banded %.4f (%.3f)  random %.3f  banded_i64 %.4f (%.3f)  ok %s' % ('$v', o['gemv_banded']['kernel_ms'], o['gemv_banded']['frac'], o['gemv']['kernel_ms'], o['gemv_banded_i64']['kernel_ms'], o['gemv_banded_i64']['frac'], all(o[k]['check']['ok'] for k in ('gemv_banded', 'gemv', 'gemv_banded_i64'))))"
  done
done
