#!/bin/bash
# round-3: block-level 1-D stencil as the default (every radius), parity of
# the stencil tests, the C++ suite (mhp stencils), bench stencil1d
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_elementwise.py tests/test_gpu_configs.py tests/test_gpu_comm.py tests/test_cpp_shp.py -m gpu -q -x -k "stencil or halo or suite" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03q_t.log 2>&1 || { tail -30 gpurun_out/r03q_t.log; exit 1; }
tail -1 gpurun_out/r03q_t.log
for i in 1 2; do for b in 1 0; do
  DRHIP_ST1D_BLK=$b timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --only-ops stencil1d > gpurun_out/r03q_b.json 2>gpurun_out/r03q_b.err || { tail gpurun_out/r03q_b.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r03q_b.json')); v=d['ops']['stencil1d']; print('blk=$b', round(v['kernel_ms'],4), round(v['frac'],4), v['check']['ok'])"
done; done
