#!/bin/bash
# round 5, pass f: template scan A/B #3, then the banded C4 SpMV alone at HEAD:
# rocprofv3 kernel trace + stats (the trace CSV carries the scratch size per
# work-item) and the FETCH_SIZE / WRITE_SIZE PMC passes
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/archive/r05/tscan3_ab.sh || exit 1
rm -rf gpurun_out/prof_r05_banded
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_r05_banded" -o prof --output-format csv \
  -- python3 "$R/bench.py" --steps 20 --warmup 3 --no-cpu-baseline --only-ops gemv_banded --log2n 24 \
  > gpurun_out/r05f_banded_bench.json 2> gpurun_out/r05f_banded_prof.log || { tail -20 gpurun_out/r05f_banded_prof.log; exit 1; }
cp "$(find gpurun_out/prof_r05_banded -name "*kernel_stats.csv" | head -1)" gpurun_out/r05f_kernel_stats_banded.csv
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/prof_r05_banded/**/*kernel_trace.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if "spmv" in r["Kernel_Name"]]
keys = [k for k in rows[0].keys() if "Scratch" in k or "Private" in k or "VGPR" in k or "LDS" in k]
print("spmv launches", len(rows), {k: rows[0][k] for k in keys})
ds = sorted(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows)
print("spmv ns min/median", ds[0], ds[len(ds) // 2])
PY
head -5 gpurun_out/r05f_kernel_stats_banded.csv | cut -c1-200
BENCH_ARGS="--only-ops gemv_banded --log2n 24" bash tools/pmc.sh > /dev/null || exit 1
cp gpurun_out/pmc_summary.json gpurun_out/r05f_pmc_banded.json
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/r05f_pmc_banded.json"))
for k, v in (d.items() if isinstance(d, dict) else []):
    if "spmv" in k:
        print(k, v)
PY
