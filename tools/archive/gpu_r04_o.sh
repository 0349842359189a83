#!/bin/bash
# round 4: C++ shp suite (1 / 3 / 8 segments) after the P > 1 inclusive_scan moved to the tile scan with a device-side fold
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_cpp_shp.py tests/test_gpu_scan.py -k "shp or scan or mhp" > gpurun_out/r04o_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r04o_pytest.log; [ $rc -eq 0 ] || { grep -B5 -A60 "FAILED\|Error" gpurun_out/r04o_pytest.log | head -100; exit 1; }
