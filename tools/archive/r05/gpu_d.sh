#!/bin/bash
# round 5, pass d: the IPC probe, the flag-exchange tests, the sort
# early-publish A/B (re-run with the round-4 order intact), the default bench
# line, then the whole -m gpu suite
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for k in 0 1; do timeout -k 10 60 ./tools/ipc_probe $k || { echo "ipc_probe $k rc=$?"; }; done
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_xchg.py \
  > gpurun_out/r05d_xchg.log 2>&1; rc=$?
tail -12 gpurun_out/r05d_xchg.log; [ $rc -eq 0 ] || grep -B5 -A30 "FAILED\|Error" gpurun_out/r05d_xchg.log | head -60
for rep in 1 2 3; do
  for v in 0 1; do
    echo "rep $rep E$v $(LD_LIBRARY_PATH=$PWD/tools/r05var/sortE$v timeout -k 10 60 ./tools/sort_bench 28 5 | grep drhip)" || exit 1
  done
done
bash tools/archive/r05/spmv_minw_ab.sh || exit 1
bash tools/archive/r05/spmv_minw_ab.sh || exit 1
timeout -k 10 600 python -u bench.py > gpurun_out/r05d_bench_n1.json 2> gpurun_out/r05d_bench_n1.err || { tail -20 gpurun_out/r05d_bench_n1.err; exit 1; }
python3 tools/archive/r05/bench_summary.py gpurun_out/r05d_bench_n1.json
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/r05d_pytest_gpu.log 2>&1; rc=$?
tail -4 gpurun_out/r05d_pytest_gpu.log; [ $rc -eq 0 ] || { grep -B2 -A40 "FAILED\|Error" gpurun_out/r05d_pytest_gpu.log | head -80; exit 1; }
