#!/bin/bash
# round-3: template reduce / for_each unroll A/B (dense_bench ops)
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  for v in base ru8 ru16 fu4 fu16; do
    if [ $v = base ]; then exe=tests/cpp/bin/dense_bench; else exe=tools/var_r03/$v/dense_bench; fi
    timeout -k 10 120 $exe > gpurun_out/r03l_dense.txt 2>&1 || { cat gpurun_out/r03l_dense.txt; exit 1; }
    python3 -c "
import json
r=[]
for l in open('gpurun_out/r03l_dense.txt'):
    if l.startswith('{'):
        d=json.loads(l)
        if d.get('op') in ('enumerate_for_each','zip_for_each','reduce_zip_transform','reduce_lambda_op','vector_for_each'):
            r.append(f\"{d['op']} {d['ms']:.4f} {d['frac']:.3f} {d.get('check','')}\")
print('$v', ' | '.join(r))
"
  done
done
