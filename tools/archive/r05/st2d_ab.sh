#!/bin/bash
# round 5: 2-D stencil strip height (DRHIP_ST2D_RB) variants under
# tools/r05var/st<RB>/libdrhip.so: stencil GPU tests per variant, then three
# interleaved rounds of the bench's stencil2d kernel time
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
for v in $VARS; do
  DRHIP_LIB=$PWD/tools/r05var/$v/libdrhip.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 \
    --timeout-method thread tests -m gpu -k "stencil" > gpurun_out/st_${v}_pytest.log 2>&1 || { tail -30 gpurun_out/st_${v}_pytest.log; exit 1; }
  echo "$v parity: $(tail -1 gpurun_out/st_${v}_pytest.log)"
done
for rep in 1 2 3; do
  for v in $VARS; do
    DRHIP_LIB=$PWD/tools/r05var/$v/libdrhip.so timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 \
      --no-cpu-baseline --only-ops stencil2d --log2n 24 > gpurun_out/st_${v}_$rep.json 2> gpurun_out/st_${v}_$rep.err || { tail -20 gpurun_out/st_${v}_$rep.err; exit 1; }
    python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/st_${v}_$rep.json') if l.startswith('{')][-1])
s=d['ops']['stencil2d']
print('rep $rep $v', round(s['kernel_ms'], 4), round(s['frac'], 4), s['check']['ok'])"
  done
done
