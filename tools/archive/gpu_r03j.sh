#!/bin/bash
# round-3: scan tile size (U = 16, 4 blocks/CU) and early look-back (wave 0
# resolves the prefix under the other waves' in-tile scans) at the 128-B
# granule stride, against the shipped U = 32 early-aggregate kernel
set -o pipefail
mkdir -p gpurun_out
for i in 1 2 3; do
  for v in base u16 earlylb; do
    if [ $v = base ]; then unset DRHIP_LIB; else export DRHIP_LIB=$PWD/tools/var_r03/$v/libdrhip.so; fi
    timeout -k 10 120 python bench.py --no-cpu-baseline --only-ops c2_int32 --steps 30 > gpurun_out/r03j_ab.json 2>gpurun_out/r03j_ab.err || { tail gpurun_out/r03j_ab.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/r03j_ab.json')); o=d['ops']; print('$v', 'f32 scan', round(d['roofline']['launch_ms'],4), 'i32 scan', round(o['c2_int32']['scan_ms'],4), d['check']['ok'], o['c2_int32']['check']['ok'])"
  done
done
