#!/bin/bash
# round 4: reduce_tiles grid (blocks per CU 8 / 4 / 2 / 16) at 2^26..2^30 f32, interleaved
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
LOG2S=26,27,28,30 timeout -k 10 800 python -u tools/scan_tiles_ab.py b8=default b4=tools/abvar/rt4/libdrhip.so b2=tools/abvar/rt2/libdrhip.so b16=tools/abvar/rt16/libdrhip.so > gpurun_out/r04t_ab.txt 2>&1 || { tail -20 gpurun_out/r04t_ab.txt; exit 1; }
grep -v '^{' gpurun_out/r04t_ab.txt
