#!/bin/bash
# onesweep tile size (keys per lane): timing + stamps
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for v in kpl48 kpl64 look8; do
  echo "== $v"; LD_LIBRARY_PATH=$PWD/tools/diag/$v timeout -k 10 60 ./tools/sort_bench 28 5 | head -n 1 || exit $?
done
VARIANTS="stkpl64" bash tools/sort_stamps.sh
