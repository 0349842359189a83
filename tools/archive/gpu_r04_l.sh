#!/bin/bash
# round 4: one LSD pass at 8 vs 11 bits per digit (tools/sort_digit_probe.hip), 2^28 u32
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 ./tools/sort_digit_probe 28 | tee gpurun_out/r04l_sort_digit_probe.txt
