#!/bin/bash
# round 4: C++ shp suite (column-window gemv at 1..8 segments) + gemv bench ops + mhp suite
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_cpp_shp.py > gpurun_out/r04g_cpp.log 2>&1; rc=$?
tail -5 gpurun_out/r04g_cpp.log; [ $rc -eq 0 ] || { grep -B5 -A30 "FAILED\|Error" gpurun_out/r04g_cpp.log | tail -60; exit 1; }
timeout -k 10 300 python -u bench.py --only-ops gemv --no-cpu-baseline --steps 10 > gpurun_out/r04g_bench.json 2> gpurun_out/r04g_bench.err || { tail -30 gpurun_out/r04g_bench.err; exit 1; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/r04g_bench.json"))
for k in ("gemv_banded", "gemv"):
    o = d["ops"][k]; print(k, o["ms"], o["kernel_ms"], o["frac"], o["check"]["ok"], o["x_exchange"])
PY
