#!/bin/bash
# round 5, pass t: the C2 step in int32 against f32 through the same timed
# loop (bench.py --no-ops, --dtype i32 / f32), alternating, three rounds --
# is the int32 op's 3-4 % gap in the bench line the kernels or its place in
# the bench?
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for rep in 1 2 3; do
  for dt in f32 i32; do
    timeout -k 10 300 python -u bench.py --no-ops --no-cpu-baseline --dtype $dt --steps 20 --warmup 3 > gpurun_out/t_$dt.json 2> gpurun_out/t_$dt.err || { tail -5 gpurun_out/t_$dt.err; exit 1; }
    python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/t_$dt.json') if l.startswith('{')][-1])
print('rep $rep $dt', round(d['ms_per_step'],4), 'scan frac', round(d['roofline']['frac'],4), 'scan ms', round(d['roofline']['launch_ms'],4))"
  done
done
