#!/bin/bash
# round 6, pass m: C3 at config size through the general-comparator tier
# (2^31 keys, 8 segments, lambda less / greater), bit-exact vs the oracle.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06m
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_configs.py \
  -k "lambda" -m gpu -s > $O/pytest.txt 2>&1; rc=$?
echo "rc $rc: $(tail -1 $O/pytest.txt)"; grep '^{' $O/pytest.txt | cut -c1-600
exit $rc
