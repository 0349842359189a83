#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for v in base kpl8 minw4 kpl8w4 kpl32; do
  echo "== $v"; LD_LIBRARY_PATH=$PWD/tools/variants/$v timeout -k 10 60 tools/sort_bench 28 5 | head -1 || exit 1
done
