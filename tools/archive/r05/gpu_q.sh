#!/bin/bash
# round 5, pass q: drhip_free now refuses a pointer that is not a live block.
# The C++ suite on the default allocator (0 / 3 / 8 segments), then 10 runs
# on the pool with staged copies, reporting refused frees and failures.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for dc in 0 3 8; do
  a=""; [ $dc -gt 0 ] && a="--devicesCount $dc"
  out=$(timeout -k 10 300 tests/cpp/bin/shp_tests $a 2>&1) || { echo "devices $dc FAILED"; echo "$out" | grep -E "FAILED|double|exception" | head; exit 1; }
  echo "shp_tests devices $dc: $(echo "$out" | tail -1); refused frees: $(echo "$out" | grep -c 'not a live' || true)"
done
for rep in $(seq 1 10); do
  DRHIP_ALLOC=pool DRHIP_COPY=staged timeout -k 10 300 tests/cpp/bin/shp_tests > gpurun_out/q_pool.txt 2>&1; rc=$?
  [ $rc -ge 124 ] && { echo "rc $rc"; exit $rc; }
  echo "pool rep $rep rc $rc: refused frees $(grep -c 'not a live' gpurun_out/q_pool.txt || true); $(grep -E 'FAILED' gpurun_out/q_pool.txt | tr '\n' ' ')"
done
