#!/bin/bash
# Two separate PMC passes (FETCH_SIZE, WRITE_SIZE) over a short bench run.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
export TMPDIR=/tmp
rm -rf gpurun_out/pmc_fetch gpurun_out/pmc_write
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$R/gpurun_out/pmc_fetch" -o pmc --output-format csv \
  -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/pmc_fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d "$R/gpurun_out/pmc_write" -o pmc --output-format csv \
  -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/pmc_write.log 2>&1 || exit $?
python3 tools/pmc_summary.py gpurun_out/pmc_fetch gpurun_out/pmc_write > gpurun_out/pmc_summary.json
cat gpurun_out/pmc_summary.json
