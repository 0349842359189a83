#!/bin/bash
# round 4: reduce A/B (two-level counter / flat counter / two-kernel), then the strong bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/reduce_ab.py grouped=default flat=tools/abvar/reduce_flat/libdrhip.so twokernel=tools/abvar/reduce_2k/libdrhip.so 2>&1 | tee gpurun_out/r04e_reduce_ab.txt
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_reduce.py > gpurun_out/r04e_pytest.log 2>&1 || { tail -30 gpurun_out/r04e_pytest.log; exit 1; }
tail -2 gpurun_out/r04e_pytest.log
timeout -k 10 300 python -u bench.py --only-ops c2_strong --no-cpu-baseline --steps 20 > gpurun_out/r04e_bench.json 2> gpurun_out/r04e_bench.err || { tail -30 gpurun_out/r04e_bench.err; exit 1; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/r04e_bench.json"))
c = d["ops"]["c2_strong"]; q = c["per_rank_of_8"]
print("headline", d["ms_per_step"], "reduce", d["ops"]["reduce"]["ms"], "strong", c["ms"], c.get("graph_ms"),
      "rank8", q["ms"], q.get("graph_ms"), q["reduce_kernel_ms"], q["scan_kernel_ms"], "pred", c["predicted_speedup_8"])
PY
