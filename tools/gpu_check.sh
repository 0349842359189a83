#!/bin/bash
# GPU round: parity tests, bench, rocprof kernel-trace summary.
# Each GPU step has its own time limit; a fault/abort/timeout ends the script.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
mkdir -p gpurun_out
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
STEPS=${STEPS:-10}
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest tests -m gpu -q --maxfail 30 --timeout 120 \
    --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
  ok $rc || exit $rc
fi
timeout -k 10 300 python -u bench.py --steps $STEPS --warmup 3 ${BENCH_ARGS} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench.log; [ $rc -eq 0 ] || exit $rc
if [ -z "$SKIP_PROF" ]; then
  export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o run --output-format csv \
    -- python3 "$R/bench.py" --steps $STEPS --warmup 3 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/prof.log 2>&1
  rc=$?; echo "rocprof rc=$rc"; tail -3 gpurun_out/prof.log; [ $rc -eq 0 ] || exit $rc
  find gpurun_out/prof -name '*stats*' | head
fi
