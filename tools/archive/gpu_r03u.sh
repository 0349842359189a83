#!/bin/bash
# round-3: bench.py's N = 2 path rehearsed on one GPU (gloo transport),
# including the host-side (gloo) wait around rank 0's one-process run
set -o pipefail
mkdir -p gpurun_out
SORT_LOG2N=26 bash tools/bench_2rank_1gpu.sh > gpurun_out/r03u_2rank.log 2>&1 || { tail -40 gpurun_out/r03u_2rank.log; exit 1; }
grep "^{" gpurun_out/r03u_2rank.log | tail -1 > gpurun_out/r03u_2rank.json
python3 -c "
import json; d=json.load(open('gpurun_out/r03u_2rank.json'))
print('n_gpus', d['n_gpus'], 'check', d['check'], 'combine', d['config']['combine'])
for k,v in d['ops'].items():
    c = v.get('check')
    print(k, c.get('ok') if isinstance(c, dict) else c, v.get('error', '')[:200] if isinstance(v.get('error'), str) else '')
"
