#!/bin/bash
# round 4: C++ blocking-call overhead by sync mode; sort parity at default NT=256
set -o pipefail
mkdir -p gpurun_out
for m in spin auto yield spin; do
  DRHIP_SYNC=$m timeout -k 10 120 ./tests/cpp/bin/shp_bench --overhead 0 | grep '^{' | tee -a gpurun_out/r04h_overhead.txt || exit 1
done
bash tools/sort_parity.sh
