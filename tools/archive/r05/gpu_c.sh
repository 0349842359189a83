#!/bin/bash
# round 5, pass c: new parity tests, the A/Bs (SpMV speculative window,
# template scan, sort early publish), then the whole -m gpu suite and smoke()
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread \
  tests/test_gpu_configs.py tests/test_gpu_scan.py -k "cpp_dropin or empty_segment or graph_holds or greater" \
  > gpurun_out/r05c_new.log 2>&1; rc=$?
tail -15 gpurun_out/r05c_new.log; [ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" gpurun_out/r05c_new.log | head -120; exit 1; }
for dc in 0 3 8; do
  a=""; [ $dc -gt 0 ] && a="--devicesCount $dc"
  timeout -k 10 300 tests/cpp/bin/shp_tests_lbx $a > gpurun_out/r05c_lbx_$dc.log 2>&1 || { tail -30 gpurun_out/r05c_lbx_$dc.log; exit 1; }
  echo "shp_tests_lbx devices $dc: $(tail -1 gpurun_out/r05c_lbx_$dc.log)"
done
bash tools/archive/r05/tscan_ab.sh || exit 1
bash tools/archive/r05/spmv_spec_ab.sh || exit 1
bash tools/archive/r05/sort_early_ab.sh || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/r05c_pytest_gpu.log 2>&1; rc=$?
tail -4 gpurun_out/r05c_pytest_gpu.log; [ $rc -eq 0 ] || { grep -B2 -A40 "FAILED\|Error" gpurun_out/r05c_pytest_gpu.log | head -80; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1
