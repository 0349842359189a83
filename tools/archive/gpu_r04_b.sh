#!/bin/bash
# round 4: C2 strong scaling bench line (debug of an empty first run)
set -o pipefail
mkdir -p gpurun_out
env | grep -E "^(RANK|WORLD_SIZE|LOCAL_RANK|MASTER|PYTHON)" || true; which python; python --version
timeout -k 10 300 python -u -X faulthandler bench.py --only-ops c2_strong --no-cpu-baseline --steps 20 > gpurun_out/r04b_bench.json 2> gpurun_out/r04b_bench.err
echo "bench rc=$?"
tail -30 gpurun_out/r04b_bench.err; wc -c gpurun_out/r04b_bench.json
python - <<'PY'
import json
d = json.load(open("gpurun_out/r04b_bench.json"))
print("headline", d["value"], d["ms_per_step"], d["roofline"]["frac"])
print(json.dumps(d["ops"]["c2_strong"], indent=1))
PY
