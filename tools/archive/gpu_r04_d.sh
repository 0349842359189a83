#!/bin/bash
# round 4: single-pass reduce parity, mhp suite widening (1-4 MPI ranks),
# C2 strong with HIP-graph steps
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_reduce.py tests/test_gpu_comm.py tests/test_gpu_configs.py -k "reduce or dot or comm or c2" > gpurun_out/r04d_pytest.log 2>&1 || { tail -40 gpurun_out/r04d_pytest.log; exit 1; }
tail -3 gpurun_out/r04d_pytest.log
true
timeout -k 10 300 python -u bench.py --only-ops c2_strong --no-cpu-baseline --steps 20 > gpurun_out/r04d_bench.json 2> gpurun_out/r04d_bench.err || { tail -30 gpurun_out/r04d_bench.err; exit 1; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/r04d_bench.json"))
print("headline", d["value"], d["ms_per_step"], d["roofline"]["frac"], d["ops"]["reduce"])
print(json.dumps(d["ops"]["c2_strong"], indent=1))
PY
