#!/bin/bash
# onesweep passes 1-3: AGG published from the per-wave counts before the
# digit scan (DRHIP_SORT_EARLY_PUB=1) vs after it (0): sort parity with the
# variant, then three interleaved rounds of tools/sort_bench 2^28 u32
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
DRHIP_LIB=$PWD/tools/r05var/sortE1/libdrhip.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 \
  --timeout-method thread tests/test_gpu_sort.py -m gpu > gpurun_out/r05_sortE1_pytest.log 2>&1 || { tail -30 gpurun_out/r05_sortE1_pytest.log; exit 1; }
echo "sortE1 parity: $(tail -1 gpurun_out/r05_sortE1_pytest.log)"
for rep in 1 2 3; do
  for v in 0 1; do
    echo "rep $rep E$v $(LD_LIBRARY_PATH=$PWD/tools/r05var/sortE$v timeout -k 10 60 ./tools/sort_bench 28 5 | grep drhip)" || exit 1
  done
done
