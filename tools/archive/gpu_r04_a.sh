#!/bin/bash
# round 4, first GPU call: the C5 2-D config test, then C2 strong scaling
# (2^30 total + the per-rank step of N = 8 with a one-rank RCCL combine)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 280 --timeout-method thread \
  tests/test_gpu_configs.py -k "stencil2d_2pow16" > gpurun_out/r04a_pytest.log 2>&1 || { tail -30 gpurun_out/r04a_pytest.log; exit 1; }
tail -3 gpurun_out/r04a_pytest.log
timeout -k 10 300 python -u bench.py --only-ops c2_strong --no-cpu-baseline --steps 20 > gpurun_out/r04a_bench.json 2> gpurun_out/r04a_bench.err || { tail -30 gpurun_out/r04a_bench.err; exit 1; }
python - <<'EOF'
import json
d = json.load(open("gpurun_out/r04a_bench.json"))
print("headline", d["value"], d["ms_per_step"], d["roofline"]["frac"])
print(json.dumps(d["ops"]["c2_strong"], indent=1))
EOF
