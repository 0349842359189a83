#!/bin/bash
# round-3: 2-D strip stencil with wave-edge columns through LDS (default)
# vs global edge loads (ldse0); parity first
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_elementwise.py tests/test_gpu_configs.py tests/test_cpp_shp.py -m gpu -q -x -k "stencil2d or stencil_2d or 8192 or suite" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03r_t.log 2>&1 || { tail -30 gpurun_out/r03r_t.log; exit 1; }
tail -1 gpurun_out/r03r_t.log
for i in 1 2 3; do for v in ldse1 ldse0; do
  if [ $v = ldse1 ]; then unset DRHIP_LIB; else export DRHIP_LIB=$PWD/tools/var_r03/$v/libdrhip.so; fi
  timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --only-ops stencil2d > gpurun_out/r03r_b.json 2>gpurun_out/r03r_b.err || { tail gpurun_out/r03r_b.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r03r_b.json')); v=d['ops']['stencil2d']; print('$v', round(v['kernel_ms'],4), round(v['frac'],4), v['check']['ok'])"
done; done
