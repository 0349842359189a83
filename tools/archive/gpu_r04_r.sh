#!/bin/bash
# round 4: N = 2 bench rehearsal (two ranks on one GPU over gloo) at HEAD
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
bash tools/bench_2rank_1gpu.sh > gpurun_out/r04r_rehearsal.json 2> gpurun_out/r04r_rehearsal.err || { tail -30 gpurun_out/r04r_rehearsal.err; exit 1; }
python3 - <<'PY'
import json
d = json.loads([l for l in open("gpurun_out/r04r_rehearsal.json").read().splitlines() if l.startswith("{")][-1])
print("n_gpus", d["n_gpus"], "check", d["check"], "combine", d["config"]["combine"])
for k, v in d["ops"].items():
    c = v.get("check")
    print(k, c.get("ok") if isinstance(c, dict) else c)
PY
