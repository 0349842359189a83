#!/bin/bash
# round 4: default bench line at HEAD (roofline.traffic from profiles/r04d_pmc_summary.json)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py > gpurun_out/r04f_bench_n1.json 2> gpurun_out/r04f_bench_n1.err || { tail -20 gpurun_out/r04f_bench_n1.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/r04f_bench_n1.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['roofline'],d['cpu_baseline']['value'],d['cpu_baseline']['cores'])"
