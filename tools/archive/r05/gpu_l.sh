#!/bin/bash
# round 5, pass l: stress the template scan's parity (the intermittent
# ScanNonCommutative failure of pass j): the default build (epoch statuses)
# and e0 (per-call reset), the filtered test 10x and the whole suite 3x at
# 0 and 3 segments each; a failing run prints its case (element size, n,
# input intact, first differing element)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for v in shp_tests shp_tests_e0; do
  nf=0
  for rep in $(seq 1 10); do
    timeout -k 10 300 tests/cpp/bin/$v --filter ScanNonCommutative > gpurun_out/l_$v.txt 2>&1; rc=$?
    [ $rc -ge 124 ] && { echo "$v rc $rc"; cat gpurun_out/l_$v.txt; exit $rc; }
    [ $rc -ne 0 ] && { nf=$((nf+1)); echo "$v filtered rep $rep FAILED:"; grep -E "failed|noncommutative_case" gpurun_out/l_$v.txt | head -8; }
  done
  echo "$v filtered: $nf of 10 failed"
  for dc in 0 3; do
    for rep in 1 2 3; do
      a=""; [ $dc -gt 0 ] && a="--devicesCount $dc"
      timeout -k 10 300 tests/cpp/bin/$v $a > gpurun_out/l_$v.txt 2>&1; rc=$?
      [ $rc -ge 124 ] && { echo "$v rc $rc"; exit $rc; }
      echo "$v devices $dc rep $rep rc $rc: $(grep -E 'FAILED|noncommutative_case|tests,' gpurun_out/l_$v.txt | head -6 | tr '\n' ' ')"
    done
  done
done
