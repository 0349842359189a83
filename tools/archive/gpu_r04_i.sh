#!/bin/bash
# round 4: fused gathered scan parity, c2_strong with it, 2-rank N > 1 rehearsal (overlapped halos, window gemv, merge-into sort)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_scan.py tests/test_gpu_sort.py -k "gathered or merge" > gpurun_out/r04i_pytest.log 2>&1 || { tail -30 gpurun_out/r04i_pytest.log; exit 1; }
tail -2 gpurun_out/r04i_pytest.log
timeout -k 10 300 python -u bench.py --only-ops c2_strong --no-cpu-baseline --steps 20 > gpurun_out/r04i_bench.json 2> gpurun_out/r04i_bench.err || { tail -30 gpurun_out/r04i_bench.err; exit 1; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/r04i_bench.json"))
c = d["ops"]["c2_strong"]; q = c["per_rank_of_8"]
print("headline", d["ms_per_step"], "strong", c["ms"], c.get("graph_ms"), "rank8", q["ms"], q.get("graph_ms"),
      q["reduce_kernel_ms"], q["scan_kernel_ms"], "nocomb", q["ms_without_combine"], q["graph_ms_without_combine"],
      "pred", c["predicted_speedup_8"], c["check"]["ok"], q["check"]["ok"], q.get("graph_error"))
PY
bash tools/bench_2rank_1gpu.sh > gpurun_out/r04i_rehearsal.json 2> gpurun_out/r04i_rehearsal.err; echo "rehearsal rc=$?"
python - <<'PY'
import json
for l in open("gpurun_out/r04i_rehearsal.json"):
    if l.startswith("{"):
        d = json.loads(l)
        print("N2 rehearsal", d["value"], d["check"]["ok"], {k: v.get("check", {}).get("ok") for k, v in d["ops"].items() if isinstance(v, dict)})
PY
