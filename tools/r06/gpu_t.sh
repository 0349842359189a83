#!/bin/bash
# round 6, pass t: the sort under skewed digits with the wave-uniform fast
# paths (u1: ranking + pre-pass counts; u1h: + every position counted in the
# pre-pass; u1n: + the passes' next-digit count) vs base: sort parity with
# each variant, then the skew probe and the uniform bench sort, interleaved.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06t
mkdir -p $O
for v in u1 u1h u1n; do
  DRHIP_LIB=$PWD/tools/var6/$v/libdrhip.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 \
    --timeout-method thread tests/test_gpu_sort.py -m gpu > $O/${v}_pytest.txt 2>&1; rc=$?
  echo "$v parity rc $rc: $(tail -1 $O/${v}_pytest.txt)"
  [ $rc -ne 0 ] && { grep -E "FAILED|Error" $O/${v}_pytest.txt | tail -10; exit $rc; }
done
for rep in 1 2; do
  for v in base u1 u1h u1n; do
    if [ $v = base ]; then L=$PWD/distributed-ranges_amd/libdrhip.so; else L=$PWD/tools/var6/$v/libdrhip.so; fi
    echo "== rep $rep $v"
    DRHIP_LIB=$L timeout -k 10 300 python3 tools/r06/sort_skew_probe.py 2>&1 | grep -v amdgpu.ids | tee $O/skew_${v}_$rep.txt || exit 1
  done
done
