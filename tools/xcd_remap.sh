#!/bin/bash
# XCD-aware block order on/off for the 2-D stencil and the CSR SpMV, then
# their parity tests (remap on)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for r in 1 0 1; do
  echo "== DRHIP_XCD_REMAP=$r"
  DRHIP_XCD_REMAP=$r timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline \
    --only-ops ${OPS:-stencil2d,gemv_banded,gemv} > gpurun_out/xcd_$r.log 2>&1 || exit $?
  python3 - "gpurun_out/xcd_$r.log" <<'PY'
import json, sys
line = [l for l in open(sys.argv[1]) if l.startswith("{")][-1]
ops = json.loads(line)["ops"]
for k, v in ops.items():
    print(f'{k:12s} kernel_ms {v.get("kernel_ms", v.get("ms")):.4f} frac {v.get("frac", 0):.4f} check {v.get("check", {}).get("ok")}')
PY
done
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -k "spmv or gemv or stencil or c4 or c5" > gpurun_out/pytest_xcd.log 2>&1
rc=$?; tail -n 2 gpurun_out/pytest_xcd.log; exit $rc
