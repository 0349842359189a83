#!/bin/bash
# round 4: drhip_reduce grid (blocks per CU 8 / 4 / 2) at 2^27 and 2^30 f32, interleaved
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/reduce_ab.py b8=default b4=tools/abvar/rd4/libdrhip.so b2=tools/abvar/rd2/libdrhip.so > gpurun_out/r04u_ab.txt 2>&1 || { tail -20 gpurun_out/r04u_ab.txt; exit 1; }
grep -v '^{' gpurun_out/r04u_ab.txt
