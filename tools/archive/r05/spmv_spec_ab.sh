#!/bin/bash
# banded / random C4 SpMV (2^26 rows) under the speculative x window knob
# DRHIP_SPMV_SPEC = 0 (min/max window only) / 1 (speculative, min/max on a
# miss) / 2 (speculative, global gathers on a miss): parity of each variant
# (the gemv tests), then three interleaved rounds of bench kernel times
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in 0 1 2; do
  DRHIP_LIB=$PWD/tools/r05var/spec$v/libdrhip.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 \
    --timeout-method thread tests -m gpu -k "gemv or spmv" > gpurun_out/r05_spec${v}_pytest.log 2>&1 || { tail -30 gpurun_out/r05_spec${v}_pytest.log; exit 1; }
  echo "spec$v parity: $(tail -1 gpurun_out/r05_spec${v}_pytest.log)"
done
for rep in 1 2 3; do
  for v in 0 1 2; do
    DRHIP_LIB=$PWD/tools/r05var/spec$v/libdrhip.so timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 \
      --no-cpu-baseline --only-ops gemv --log2n 24 > gpurun_out/r05_spec${v}_$rep.json 2> gpurun_out/r05_spec${v}_$rep.err || { tail -20 gpurun_out/r05_spec${v}_$rep.err; exit 1; }
    python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/r05_spec${v}_$rep.json') if l.startswith('{')][-1])
b, r = d['ops']['gemv_banded'], d['ops']['gemv']
print('rep $rep spec$v banded', round(b['kernel_ms'], 4), round(b['frac'], 4), b['check']['ok'], 'random', round(r['kernel_ms'], 3), r['check']['ok'])"
  done
done
