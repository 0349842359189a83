#!/bin/bash
# round-3 closing check at HEAD: the whole -m gpu suite and smoke()
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/r03_pytest_gpu_head.txt 2>&1
rc=$?; tail -3 gpurun_out/r03_pytest_gpu_head.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_smoke.txt 2>&1 || { cat gpurun_out/r03_smoke.txt; exit 1; }
tail -1 gpurun_out/r03_smoke.txt
