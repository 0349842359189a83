#!/bin/bash
# round 4: kernel timeline of C2 strong (2^30) and its per-rank-of-8 step
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/r04c_prof -o trace -- \
  python -u bench.py --only-ops c2_strong --no-cpu-baseline --steps 20 > gpurun_out/r04c_bench.json 2> gpurun_out/r04c_bench.err
echo "rc=$?"
tail -5 gpurun_out/r04c_bench.err
head -c 300 gpurun_out/r04c_bench.json
find gpurun_out/r04c_prof -name "*.csv" | head
