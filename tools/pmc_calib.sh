#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration (tools/pmc_calib.hip: known byte counts)
# and the C4 SpMV split by matrix kind + the sort, one counter per pass.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 60 ./tools/pmc_calib > gpurun_out/calib_time.log 2>&1 || exit $?
cat gpurun_out/calib_time.log
for c in FETCH_SIZE WRITE_SIZE; do
  rm -rf gpurun_out/calib_$c
  timeout -s KILL 90 rocprofv3 --pmc $c -d "$R/gpurun_out/calib_$c" -o pmc --output-format csv \
    -- "$R/tools/pmc_calib" > gpurun_out/calib_$c.log 2>&1 || exit $?
done
for op in gemv_banded gemv_random sort; do
  for c in FETCH_SIZE WRITE_SIZE; do
    rm -rf gpurun_out/pmc_${op}_$c
    timeout -s KILL 180 rocprofv3 --pmc $c -d "$R/gpurun_out/pmc_${op}_$c" -o pmc --output-format csv \
      -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --only-ops $op --log2n 20 \
      > gpurun_out/pmc_${op}_$c.log 2>&1 || exit $?
  done
done
python3 tools/pmc_summary.py --calib gpurun_out > gpurun_out/pmc_calib_summary.json
cat gpurun_out/pmc_calib_summary.json
