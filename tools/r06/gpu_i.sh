#!/bin/bash
# round 6, pass i: the dot kernel vs the relative placement of x and y
# (tools/r06/dot_offsets.py), and the bench's own dot op layout.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06i
mkdir -p $O
timeout -k 10 300 python3 tools/r06/dot_offsets.py 2>&1 | tee $O/dot_offsets.txt || exit 1
timeout -k 10 300 python3 bench.py --only-ops dot --log2n 24 --steps 20 --warmup 20 --no-cpu-baseline > $O/dot_alone.json 2> $O/dot_alone.err || exit 1
python3 -c "
import json; o=json.load(open('$O/dot_alone.json'))['ops']['dot']
print('bench dot alone: kernel %.4f loop %.4f y-x %d MiB' % (o['kernel_ms'], o['loop_kernel_ms'], o['y_minus_x_bytes'] >> 20))"
# the merge-sort tier with 1024-thread block-sort tiles: the C++ suites, then
# the one-process bench (sort_lambda_cmp)
timeout -k 10 600 python -u -m pytest tests/test_cpp_shp.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_cpp.txt 2>&1; rc=$?
echo "pytest cpp rc $rc: $(tail -1 $O/pytest_cpp.txt)"
[ $rc -ne 0 ] && { grep -E "FAILED|Error|MISMATCH|mismatch" $O/pytest_cpp.txt | head -20; exit $rc; }
timeout -k 10 300 tests/cpp/bin/shp_bench --devices 0 --reps 5 > $O/shp_bench.json 2>&1; echo "shp_bench rc $?"; tail -c 1200 $O/shp_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_shp -o shp --output-format csv -- tests/cpp/bin/shp_bench --devices 0 --reps 5 > $O/prof_shp.log 2>&1; echo "rocprof shp_bench rc $?"
