#!/bin/bash
# round 4: rocprofv3 kernel stats of the headline alone (2^30 f32, --no-ops),
# so the roofline kernel's average is over 2^30 launches only
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/prof_r04c
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_r04c" -o prof --output-format csv \
  -- python3 "$R/bench.py" --steps 20 --warmup 3 --no-cpu-baseline --no-ops > gpurun_out/r04c_bench_noops.json 2> gpurun_out/prof_r04c.log || { tail -20 gpurun_out/prof_r04c.log; exit 1; }
f=$(find gpurun_out/prof_r04c -name "*kernel_stats.csv" | head -1)
cp "$f" gpurun_out/r04c_kernel_stats_bench_2p30_f32.csv
grep drhip gpurun_out/r04c_kernel_stats_bench_2p30_f32.csv | cut -c1-60,400-
