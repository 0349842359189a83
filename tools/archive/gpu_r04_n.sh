#!/bin/bash
# round 4: wave-part tile-prefix scan at 2 vectors per thread (blockIdx order) with the grouped small-tile
# reduce -- parity (tile tests), then A/B over 2^26..2^30 against U = 32 (counter order) and the ungrouped reduce
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_scan.py -k "tiles or gathered" > gpurun_out/r04n_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r04n_pytest.log; [ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" gpurun_out/r04n_pytest.log | head -80; exit 1; }
LOG2S=26,27,28,29,30 timeout -k 10 800 python -u tools/scan_tiles_ab.py wave2d=default w32n=tools/abvar/w32n/libdrhip.so w16n=tools/abvar/w16n/libdrhip.so wave32=tools/abvar/wave_u32/libdrhip.so > gpurun_out/r04n_ab.txt 2>&1 || { tail -20 gpurun_out/r04n_ab.txt; exit 1; }
grep -v '^{' gpurun_out/r04n_ab.txt
