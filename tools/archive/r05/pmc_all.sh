#!/bin/bash
# round 5: FETCH_SIZE / WRITE_SIZE over every op of the default bench at HEAD
# (two separate PMC passes, as tools/pmc.sh, with room for the whole bench)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
export TMPDIR=/tmp
rm -rf gpurun_out/pmca_fetch gpurun_out/pmca_write
timeout -s KILL 500 rocprofv3 --pmc FETCH_SIZE -d "$R/gpurun_out/pmca_fetch" -o pmc --output-format csv \
  -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmca_fetch.log 2>&1 || exit $?
timeout -s KILL 500 rocprofv3 --pmc WRITE_SIZE -d "$R/gpurun_out/pmca_write" -o pmc --output-format csv \
  -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmca_write.log 2>&1 || exit $?
python3 tools/pmc_summary.py gpurun_out/pmca_fetch gpurun_out/pmca_write > gpurun_out/r05_pmc_summary_all_ops.json
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/r05_pmc_summary_all_ops.json"))
for k, v in d["kernels"].items():
    if k.startswith("void drhip") or "shp::" in k:
        print(k[:80], v)
PY
