#!/bin/bash
# ad-hoc GPU pass: chosen -m gpu test files, the N=2 rehearsal, a bench subset
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest ${TESTS:-tests/test_gpu_reduce.py tests/test_gpu_sort.py tests/test_cpp_shp.py} -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/pytest_a.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_a.log; [ $rc -eq 0 ] || exit $rc
if [ -n "$REHEARSE" ]; then
  bash tools/bench_2rank_1gpu.sh > gpurun_out/bench2.log 2>&1
  rc=$?; tail -c 3000 gpurun_out/bench2.log; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "$OPS" ]; then
  timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --only-ops $OPS --no-cpu-baseline > gpurun_out/bench_a.log 2>&1
  rc=$?; tail -c 2500 gpurun_out/bench_a.log; [ $rc -eq 0 ] || exit $rc
fi
exit 0
