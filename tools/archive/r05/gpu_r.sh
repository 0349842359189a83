#!/bin/bash
# round 5, pass r: which part of the C++ suite the pool corruption needs.
# pool + staged copies (the strongest amplifier), 10 runs per filter
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for flt in ScanNonCommutative Scan ShpExtra ""; do
  nf=0
  for rep in $(seq 1 10); do
    a=""; [ -n "$flt" ] && a="--filter $flt"
    DRHIP_ALLOC=pool DRHIP_COPY=staged timeout -k 10 300 tests/cpp/bin/shp_tests $a > gpurun_out/r_cur.txt 2>&1; rc=$?
    [ $rc -ge 124 ] && { echo "rc $rc"; exit $rc; }
    [ $rc -ne 0 ] && nf=$((nf+1))
  done
  echo "filter '${flt}': $nf of 10 failed; last run: $(grep -E 'FAILED|tests,' gpurun_out/r_cur.txt | tr '\n' ' ')"
done
