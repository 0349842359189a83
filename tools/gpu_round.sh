#!/bin/bash
# One GPU pass: chosen pytest files (-m gpu), then bench.py; each step under
# its own time limit, stop at the first failure.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TESTS=${TESTS:-tests}
if [ -n "$TESTS" ] && [ "$TESTS" != "none" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest $TESTS -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|passed|failed|Error" gpurun_out/pytest_gpu.log | tail -15
  [ $rc -eq 0 ] || exit $rc
fi
if [ -z "$SKIP_BENCH" ]; then
  timeout -k 10 400 python -u bench.py --steps ${STEPS:-10} --warmup 3 ${BENCH_ARGS} > gpurun_out/bench.log 2>&1
  rc=$?; echo "bench rc=$rc"; tail -c 6000 gpurun_out/bench.log; exit $rc
fi
