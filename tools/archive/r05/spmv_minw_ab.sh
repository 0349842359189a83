#!/bin/bash
# banded / random C4 SpMV (2^26 rows) with the speculative window at 8 / 7 / 6
# waves per SIMD for the 4-byte kernel (DRHIP_SPMV_MINW_4B: 64 VGPRs + 10
# spilled / 72 + 2 / 74 + 0): parity per variant, three interleaved rounds
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in 8 7 6; do
  DRHIP_LIB=$PWD/tools/r05var/spmvw$v/libdrhip.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 \
    --timeout-method thread tests -m gpu -k "gemv or spmv" > gpurun_out/r05_spmvw${v}_pytest.log 2>&1 || { tail -30 gpurun_out/r05_spmvw${v}_pytest.log; exit 1; }
  echo "spmvw$v parity: $(tail -1 gpurun_out/r05_spmvw${v}_pytest.log)"
done
for rep in 1 2 3; do
  for v in 8 7 6; do
    DRHIP_LIB=$PWD/tools/r05var/spmvw$v/libdrhip.so timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 \
      --no-cpu-baseline --only-ops gemv --log2n 24 > gpurun_out/r05_spmvw${v}_$rep.json 2> gpurun_out/r05_spmvw${v}_$rep.err || { tail -20 gpurun_out/r05_spmvw${v}_$rep.err; exit 1; }
    python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/r05_spmvw${v}_$rep.json') if l.startswith('{')][-1])
b, r = d['ops']['gemv_banded'], d['ops']['gemv']
print('rep $rep spmvw$v banded', round(b['kernel_ms'], 4), round(b['frac'], 4), b['check']['ok'], 'random', round(r['kernel_ms'], 3), r['check']['ok'])"
  done
done
