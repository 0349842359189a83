#!/bin/bash
# round 6, pass ac: FETCH_SIZE / WRITE_SIZE over every op of the default bench at the final HEAD (two separate PMC passes)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
export TMPDIR=/tmp
O=gpurun_out/r06ac
mkdir -p $O
rm -rf $O/pmc_fetch $O/pmc_write
timeout -s KILL 500 rocprofv3 --pmc FETCH_SIZE -d "$R/$O/pmc_fetch" -o pmc --output-format csv \
  -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline > $O/pmc_fetch.log 2>&1 || exit $?
echo "fetch pass done"
timeout -s KILL 500 rocprofv3 --pmc WRITE_SIZE -d "$R/$O/pmc_write" -o pmc --output-format csv \
  -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline > $O/pmc_write.log 2>&1 || exit $?
echo "write pass done"
python3 tools/pmc_summary.py $O/pmc_fetch $O/pmc_write > $O/r06ac_pmc_summary_all_ops.json
python3 - <<PY
import json
d = json.load(open("$O/r06ac_pmc_summary_all_ops.json"))
for k, v in d["kernels"].items():
    if k.startswith("void drhip") or "drhip::" in k:
        print(k[:80], {a: b for a, b in v.items() if "bytes" in a or "launches" in a})
PY
