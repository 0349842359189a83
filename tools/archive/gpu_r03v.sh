#!/bin/bash
# round-3: onesweep look-back width (predecessors per round trip) with the
# same-XCD status copy: 4 (shipped) vs 2 / 8
set -o pipefail
mkdir -p gpurun_out
for i in 1 2 3; do
  for v in look4 look2 look8; do
    if [ $v = look4 ]; then unset DRHIP_LIB; else export DRHIP_LIB=$PWD/tools/var_r03/$v/libdrhip.so; fi
    timeout -k 10 120 python bench.py --no-cpu-baseline --only-ops sort --steps 20 > gpurun_out/r03v_sort.json 2>gpurun_out/r03v_sort.err || { tail gpurun_out/r03v_sort.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/r03v_sort.json')); o=d['ops']['sort']; print('$v', 'local sort', round(o['local_sort_ms'],4), o['check']['ok'])"
  done
done
