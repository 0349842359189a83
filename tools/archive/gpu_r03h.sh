#!/bin/bash
# round-3 evidence: rocprofv3 kernel stats of the full bench (every op), then
# separate FETCH_SIZE / WRITE_SIZE PMC passes of the headline (no ops)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/prof_r03
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_r03" -o prof --output-format csv \
  -- python3 "$R/bench.py" --steps 20 --warmup 3 > gpurun_out/prof_r03.log 2>&1 || { tail -20 gpurun_out/prof_r03.log; exit 1; }
f=$(find gpurun_out/prof_r03 -name "*kernel_stats.csv" | head -1)
cp "$f" gpurun_out/r03_kernel_stats_bench.csv
head -25 gpurun_out/r03_kernel_stats_bench.csv | cut -c1-200
grep "^{" gpurun_out/prof_r03.log | tail -1 > gpurun_out/r03_bench_under_rocprof.json
BENCH_ARGS="--no-ops" bash tools/pmc.sh || exit 1
