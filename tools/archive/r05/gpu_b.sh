#!/bin/bash
# round 5, pass b: the new parity tests, the SpMV speculative-window A/B,
# then the whole -m gpu suite and smoke()
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread \
  tests/test_gpu_configs.py tests/test_gpu_scan.py -k "cpp_dropin or empty_segment or graph_holds or greater" \
  > gpurun_out/r05b_new.log 2>&1; rc=$?
tail -15 gpurun_out/r05b_new.log; [ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" gpurun_out/r05b_new.log | head -120; exit 1; }
bash tools/archive/r05/spmv_spec_ab.sh || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/r05b_pytest_gpu.log 2>&1; rc=$?
tail -4 gpurun_out/r05b_pytest_gpu.log; [ $rc -eq 0 ] || { grep -B2 -A40 "FAILED\|Error" gpurun_out/r05b_pytest_gpu.log | head -80; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1
