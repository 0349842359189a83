#!/bin/bash
# round-3: block-level 1-D stencil (wave edges through LDS) x cache policy,
# against the shipped wave-level kernel; parity first
set -o pipefail
mkdir -p gpurun_out
for b in 1; do for v in 0 1 2 3; do
  DRHIP_ST1D_BLK=$b DRHIP_ST_NT=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_elementwise.py tests/test_gpu_configs.py -m gpu -q -x -k "stencil1d or stencil_1d" --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r03p_t.log 2>&1 || { tail -30 gpurun_out/r03p_t.log; exit 1; }
  echo "blk=$b nt=$v $(tail -1 gpurun_out/r03p_t.log)"
done; done
for i in 1 2; do
  for cfg in "0 0" "1 0" "1 1" "1 2" "1 3"; do
    set -- $cfg
    DRHIP_ST1D_BLK=$1 DRHIP_ST_NT=$2 timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --only-ops stencil1d > gpurun_out/r03p_b.json 2>gpurun_out/r03p_b.err || { tail gpurun_out/r03p_b.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/r03p_b.json')); v=d['ops']['stencil1d']; print('blk=$1 nt=$2', round(v['kernel_ms'],4), round(v['frac'],4), v['check']['ok'])"
  done
done
