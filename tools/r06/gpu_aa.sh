#!/bin/bash
# round 6, pass aa: the C++ suites with the 24-/40-byte general-sort cases,
# the sort parity tests, and smoke, on the final library build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06aa
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_cpp_shp.py tests/test_gpu_sort.py \
  -m gpu > $O/pytest.txt 2>&1; rc=$?
echo "pytest rc $rc: $(tail -1 $O/pytest.txt)"
[ $rc -ne 0 ] && { grep -E "FAILED|Error|Failure" $O/pytest.txt | tail -20; exit $rc; }
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1
