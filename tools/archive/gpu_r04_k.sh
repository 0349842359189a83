#!/bin/bash
# round 4: tile-prefix scan: one-shot U = 32 vs the persistent two-tile pipeline (U = 16 / 8)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/scan_tiles_ab.py u32=default pipe16=tools/abvar/pipe_u16/libdrhip.so pipe8=tools/abvar/pipe_u8/libdrhip.so > gpurun_out/r04k_ab.txt 2>&1 || { tail -20 gpurun_out/r04k_ab.txt; exit 1; }
grep -v '^{' gpurun_out/r04k_ab.txt
