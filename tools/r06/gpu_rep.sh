#!/bin/bash
# round 6: the whole -m gpu suite twice more at the final HEAD (stability),
# stopping at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06rep
mkdir -p $O
for i in 1 2; do
  timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $O/pytest_$i.txt 2>&1; rc=$?
  echo "run $i rc $rc: $(tail -1 $O/pytest_$i.txt)"
  [ $rc -ne 0 ] && { grep -E "FAILED|Error" $O/pytest_$i.txt | tail -20; exit $rc; }
done
exit 0
