#!/bin/bash
# SpMV stream kernel: 7 waves/SIMD (68 VGPRs, shipped) vs 8 (DRHIP_SPMV_MINW=8
# variant, tools/diag/minw8), interleaved bench runs of the C4 ops
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for v in base minw8 base minw8; do
  lib=""; [ "$v" = minw8 ] && lib="$PWD/tools/diag/minw8/libdrhip.so"
  DRHIP_LIB=$lib timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline \
    --only-ops gemv_banded,gemv > gpurun_out/spmv_$v.log 2>&1 || exit $?
  python3 - "gpurun_out/spmv_$v.log" "$v" <<'PY'
import json, sys
line = [l for l in open(sys.argv[1]) if l.startswith("{")][-1]
ops = json.loads(line)["ops"]
for k in ("gemv_banded", "gemv"):
    v = ops[k]
    print(f'{sys.argv[2]:6s} {k:12s} kernel_ms {v["kernel_ms"]:.4f} frac {v["frac"]:.4f} check {v["check"]["ok"]}')
PY
done
