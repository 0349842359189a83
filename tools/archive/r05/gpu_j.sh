#!/bin/bash
# round 5, pass j: template scan TEXC (the look-back prefix folded in the
# combine, no s_pre rewrite by wave 0) and PRIO (wave 0 at s_setprio 3),
# alone and together, against the shipped form (e0).  Parity: the default C++
# suite and the t1p1 build at 0 / 3 / 8 segments; then four interleaved
# rounds of dense_bench; rocprof of e0 and t1p1.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for b in shp_tests shp_tests_t1p1; do
  for dc in 0 3 8; do
    a=""; [ $dc -gt 0 ] && a="--devicesCount $dc"
    out=$(timeout -k 10 300 tests/cpp/bin/$b $a) || { echo "$b devices $dc FAILED"; echo "$out" | grep -E "failed|FAILED|exception|noncommutative" | head -20; exit 1; }
    echo "$b devices $dc: $(echo "$out" | tail -1)"
  done
done
for rep in 1 2 3 4; do
  for v in e0 t1 p1 t1p1; do
    out=$(timeout -k 10 120 tests/cpp/bin/dense_bench_$v 15 15 10) || { echo "$v failed"; exit 1; }
    echo "rep $rep $v $(echo "$out" | grep scan_lambda_op)"
  done
done
for v in e0 t1p1; do
  rm -rf gpurun_out/r05j_prof_$v
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/r05j_prof_$v" -o run --output-format csv \
    -- tests/cpp/bin/dense_bench_$v 15 15 10 > gpurun_out/r05j_prof_$v.log 2>&1 || exit $?
  f=$(find gpurun_out/r05j_prof_$v -name '*kernel_stats.csv' | head -1)
  echo "== $v"; grep -E "lb_scan|fillBuffer" "$f" | awk -F'","' '{print substr($1,1,50), $2, $4}'
done
