#!/bin/bash
# stencil cache-policy variants (DRHIP_ST_NT 0..3), bench kernel times
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for v in 0 1 2 3 0; do
  DRHIP_ST_NT=$v timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline \
    --only-ops stencil1d,stencil2d > gpurun_out/stnt_$v.log 2>&1 || exit $?
  python3 - "gpurun_out/stnt_$v.log" "$v" <<'PY'
import json, sys
line = [l for l in open(sys.argv[1]) if l.startswith("{")][-1]
ops = json.loads(line)["ops"]
for k in ("stencil1d", "stencil2d"):
    v = ops[k]
    print(f'NT={sys.argv[2]} {k:10s} kernel_ms {v["kernel_ms"]:.4f} frac {v["frac"]:.4f} check {v["check"]["ok"]}')
PY
done
