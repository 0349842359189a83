#!/bin/bash
# round 4: reduce / dot / C2 parity after the reduce grid change, then the default bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu -k "reduce or dot or c2 or smoke" > gpurun_out/r04v_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r04v_pytest.log; [ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" gpurun_out/r04v_pytest.log | head -80; exit 1; }
timeout -k 10 600 python -u bench.py > gpurun_out/r04v_bench_n1.json 2> gpurun_out/r04v_bench_n1.err || { tail -20 gpurun_out/r04v_bench_n1.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/r04v_bench_n1.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['roofline']['frac'],{k:(v.get('check') or {}).get('ok') for k,v in d['ops'].items() if isinstance(v.get('check'),dict)})"
