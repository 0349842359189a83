#!/bin/bash
# round 6, pass j: the merge-sort tier with padded LDS tiles and 32-bit LDS
# merge paths -- the C++ suites (bit-exact vs std::stable_sort), then the
# one-process bench at 256 (default) and 1024 block-sort threads, interleaved,
# and the kernel stats of the default.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06j
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_cpp_shp.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_cpp.txt 2>&1; rc=$?
echo "pytest cpp rc $rc: $(tail -1 $O/pytest_cpp.txt)"
[ $rc -ne 0 ] && { grep -E "FAILED|Error|mismatch" $O/pytest_cpp.txt | head -20; exit $rc; }
for rep in 1 2 3; do
  for v in shp_bench shp_bench_st1024; do
    timeout -k 10 300 tests/cpp/bin/$v --devices 0 --reps 5 > $O/${v}_$rep.json 2>&1 || { tail -5 $O/${v}_$rep.json; exit 1; }
    python3 -c "
import json; d=[json.loads(l) for l in open('$O/${v}_$rep.json') if l.startswith('{')][-1]
print('rep $rep $v sort_lambda_cmp %.3f ms bad %d ok %s' % (d['sort_lambda_cmp']['ms'], d['sort_lambda_cmp']['bad'], d['check']['ok']))"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_shp -o shp --output-format csv -- tests/cpp/bin/shp_bench --devices 0 --reps 5 > $O/prof_shp.log 2>&1; echo "rocprof rc $?"
python3 - <<PY
import csv
for r in csv.DictReader(open("$O/prof_shp/shp_kernel_stats.csv")):
    if "msort" in r["Name"]:
        print("%-70s calls %4s avg_ms %.4f" % (r["Name"][:70], r["Calls"], float(r["AverageNs"]) / 1e6))
PY
