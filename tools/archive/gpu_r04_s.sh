#!/bin/bash
# round 4: FETCH_SIZE / WRITE_SIZE passes over the FULL default bench (every op), at HEAD
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
BENCH_ARGS="" bash tools/pmc.sh > /dev/null || exit 1
cp gpurun_out/pmc_summary.json gpurun_out/r04s_pmc_summary_all_ops.json
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/r04s_pmc_summary_all_ops.json"))
for k, v in d["kernels"].items():
    if "drhip" in k:
        print(k[:80], v.get("dispatches"), v.get("fetch_bytes_raw"), v.get("write_bytes_raw"), v.get("hbm_bytes_per_launch"))
PY
