#!/bin/bash
# onesweep look-back width (predecessors per round trip): timing + stamps
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for v in look8 look16; do
  echo "== $v"; LD_LIBRARY_PATH=$PWD/tools/diag/$v timeout -k 10 60 ./tools/sort_bench 28 5 | head -n 1 || exit $?
done
echo "== base"; timeout -k 10 60 ./tools/sort_bench 28 5 | head -n 1 || exit $?
VARIANTS="stlook8 stlook16" bash tools/sort_stamps.sh
