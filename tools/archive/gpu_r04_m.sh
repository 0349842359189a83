#!/bin/bash
# round 4: tile-scan in-place / counter-reset test + the scan tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_scan.py > gpurun_out/r04m_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r04m_pytest.log; [ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" gpurun_out/r04m_pytest.log | head -80; exit 1; }
