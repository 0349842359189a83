#!/bin/bash
# round-3 probes: XCD-local ping-pong copy bandwidth (L2 / Infinity Cache
# resident working sets), stencil cache-policy variants
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 tools/xcd_local_copy > gpurun_out/r03i_xcd_copy.txt 2>&1 || { cat gpurun_out/r03i_xcd_copy.txt; exit 1; }
cat gpurun_out/r03i_xcd_copy.txt
timeout -k 10 500 bash tools/stencil_nt.sh > gpurun_out/r03i_stnt.txt 2>&1 || { cat gpurun_out/r03i_stnt.txt; exit 1; }
cat gpurun_out/r03i_stnt.txt
