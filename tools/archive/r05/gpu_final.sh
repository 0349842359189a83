#!/bin/bash
# round-5 evidence at HEAD: the whole -m gpu suite, smoke(), the default bench
# line, rocprofv3 kernel stats of the full bench and of the headline alone,
# the FETCH_SIZE / WRITE_SIZE PMC passes of the headline, and the N = 2 / N = 4
# rehearsals of the bench on one GPU (gloo; the flag-slot combine over IPC)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
T=${TAG:-r05z}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1; rc=$?
tail -4 gpurun_out/${T}_pytest_gpu.log; [ $rc -eq 0 ] || { grep -B2 -A40 "FAILED\|Error" gpurun_out/${T}_pytest_gpu.log | head -80; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1
timeout -k 10 600 python -u bench.py > gpurun_out/${T}_bench_n1.json 2> gpurun_out/${T}_bench_n1.err || { tail -20 gpurun_out/${T}_bench_n1.err; exit 1; }
python3 tools/archive/r05/bench_summary.py gpurun_out/${T}_bench_n1.json
rm -rf gpurun_out/prof_${T}
timeout -s KILL 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_${T}" -o prof --output-format csv \
  -- python3 "$R/bench.py" --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/prof_${T}.log 2>&1 || { tail -20 gpurun_out/prof_${T}.log; exit 1; }
cp "$(find gpurun_out/prof_${T} -name "*kernel_stats.csv" | head -1)" gpurun_out/${T}_kernel_stats_bench.csv
head -12 gpurun_out/${T}_kernel_stats_bench.csv | cut -c1-160
rm -rf gpurun_out/prof_${T}h
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_${T}h" -o prof --output-format csv \
  -- python3 "$R/bench.py" --steps 20 --warmup 3 --no-cpu-baseline --no-ops > gpurun_out/${T}_bench_noops.json 2> gpurun_out/prof_${T}h.log || { tail -20 gpurun_out/prof_${T}h.log; exit 1; }
cp "$(find gpurun_out/prof_${T}h -name "*kernel_stats.csv" | head -1)" gpurun_out/${T}_kernel_stats_bench_2p30_f32.csv
head -6 gpurun_out/${T}_kernel_stats_bench_2p30_f32.csv | cut -c1-160
BENCH_ARGS="--no-ops" bash tools/pmc.sh > /dev/null || exit 1
cp gpurun_out/pmc_summary.json gpurun_out/${T}_pmc_summary.json
python3 - <<PY
import json
d = json.load(open("gpurun_out/${T}_pmc_summary.json"))
for k, v in d["kernels"].items():
    if "scan" in k or "reduce" in k:
        print(k[:90], v)
PY
bash tools/bench_2rank_1gpu.sh > gpurun_out/${T}_rehearsal_n2.json 2> gpurun_out/${T}_rehearsal_n2.err || { tail -30 gpurun_out/${T}_rehearsal_n2.err; exit 1; }
python3 tools/archive/r05/bench_summary.py gpurun_out/${T}_rehearsal_n2.json
NPROC=4 bash tools/bench_2rank_1gpu.sh > gpurun_out/${T}_rehearsal_n4.json 2> gpurun_out/${T}_rehearsal_n4.err || { tail -30 gpurun_out/${T}_rehearsal_n4.err; exit 1; }
python3 tools/archive/r05/bench_summary.py gpurun_out/${T}_rehearsal_n4.json
