#!/bin/bash
# round 4: tile-prefix reduce + scan parity, then the bench headline / c2_strong with it
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_scan.py tests/test_gpu_configs.py -k "tiles or gathered or c2" > gpurun_out/r04j_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r04j_pytest.log; [ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" gpurun_out/r04j_pytest.log | head -80; exit 1; }
timeout -k 10 300 python -u bench.py --only-ops c2_strong,c2_int32 --no-cpu-baseline --steps 20 > gpurun_out/r04j_bench.json 2> gpurun_out/r04j_bench.err || { tail -30 gpurun_out/r04j_bench.err; exit 1; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/r04j_bench.json"))
o = d["ops"]; c = o["c2_strong"]; q = c["per_rank_of_8"]
print("headline", d["value"], d["ms_per_step"], "scan frac", d["roofline"]["frac"], "reduce", o["reduce"]["ms"], o["reduce"]["frac"],
      "scan", o["inclusive_scan"]["ms"], "single-pass", o["inclusive_scan_single_pass"]["ms"], o["inclusive_scan_single_pass"]["frac"], d["check"])
print("c2_int32", o["c2_int32"]["ms"], o["c2_int32"]["reduce_frac"], o["c2_int32"]["scan_frac"], o["c2_int32"]["check"]["ok"])
print("strong", c["ms"], c.get("graph_ms"), "rank8", q["ms"], q.get("graph_ms"), q["reduce_kernel_ms"], q["scan_kernel_ms"],
      "nocomb", q["ms_without_combine"], q["graph_ms_without_combine"], "pred", c["predicted_speedup_8"], c["check"]["ok"], q["check"]["ok"], q.get("graph_error"))
PY
