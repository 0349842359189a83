#!/bin/bash
# round 5, pass e: the flag-exchange tests (rank processes over IPC), the
# N = 2 bench rehearsal on one GPU (gloo; the flag combine over IPC at N > 1)
# plain and with a capture failure injected on rank 1, shp_bench's new
# fp64 check, then the whole -m gpu suite
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_xchg.py \
  > gpurun_out/r05e_xchg.log 2>&1; rc=$?
tail -8 gpurun_out/r05e_xchg.log; [ $rc -eq 0 ] || { grep -B5 -A30 "FAILED\|Error" gpurun_out/r05e_xchg.log | head -80; exit 1; }
bash tools/bench_2rank_1gpu.sh > gpurun_out/r05e_rehearsal.json 2> gpurun_out/r05e_rehearsal.err || { tail -30 gpurun_out/r05e_rehearsal.err; exit 1; }
python3 tools/archive/r05/bench_summary.py gpurun_out/r05e_rehearsal.json
python3 - <<'PY'
import json
d = json.loads([l for l in open("gpurun_out/r05e_rehearsal.json") if l.startswith("{")][-1])
c = d["ops"]["c2_strong"]
print("c2_strong note", c.get("note"), "graph_error", c.get("graph_error"))
f = c.get("flags", {})
print("flags", {k: f.get(k) for k in ("ms", "graph_ms", "error", "combine")}, f.get("check", {}).get("ok"))
PY
DRHIP_BENCH_FAIL_CAPTURE_RANK=1 bash tools/bench_2rank_1gpu.sh > gpurun_out/r05e_rehearsal_fail1.json 2> gpurun_out/r05e_rehearsal_fail1.err || { tail -30 gpurun_out/r05e_rehearsal_fail1.err; exit 1; }
python3 - <<'PY'
import json
d = json.loads([l for l in open("gpurun_out/r05e_rehearsal_fail1.json") if l.startswith("{")][-1])
c = d["ops"]["c2_strong"]
print("injected: c2_strong graph_error", c.get("graph_error"), "ms", c.get("ms"), "check", c.get("check", {}).get("ok"))
f = c.get("flags", {})
print("injected: flags graph_error", f.get("graph_error"), "check", f.get("check", {}).get("ok"))
PY
bash tools/archive/r05/tscan2_ab.sh || exit 1
timeout -k 10 300 tests/cpp/bin/shp_bench --devices 0 --reps 3 | tee gpurun_out/r05e_shp_bench.json || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/r05e_pytest_gpu.log 2>&1; rc=$?
tail -4 gpurun_out/r05e_pytest_gpu.log; [ $rc -eq 0 ] || { grep -B2 -A40 "FAILED\|Error" gpurun_out/r05e_pytest_gpu.log | head -80; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1
