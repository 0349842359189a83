#!/bin/bash
# round 5, pass i: the template scan without a status reset per call
# (DR_SHP_LB_EPOCH: epoch-tagged status words, self-resetting tile counter)
# and with a DPP look-back fold (DR_SHP_LB_DPPLB), alone and together.
# Parity: the C++ suite built with the knob (ep1) and with a 3-epoch wrap
# (ep1w3: the status clear every third call) at 0 / 3 / 8 segments; then
# three interleaved rounds of dense_bench ep0 / ep1, and one rocprof pass
# of each (kernel and fill-kernel counts per call).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for b in shp_tests_ep1 shp_tests_ep1w3 shp_tests_dl1 shp_tests_ep1dl1; do
  for dc in 0 3 8; do
    a=""; [ $dc -gt 0 ] && a="--devicesCount $dc"
    out=$(timeout -k 10 300 tests/cpp/bin/$b $a) || { echo "$b devices $dc FAILED"; echo "$out" | tail -20; exit 1; }
    echo "$b devices $dc: $(echo "$out" | tail -1)"
  done
done
for rep in 1 2 3; do
  for v in ep0 ep1 dl1 ep1dl1; do
    out=$(timeout -k 10 120 tests/cpp/bin/dense_bench_$v 15 15 10) || { echo "$v failed"; exit 1; }
    echo "rep $rep $v $(echo "$out" | grep scan_lambda_op)"
  done
done
for v in ep0 ep1dl1; do
  rm -rf gpurun_out/r05i_prof_$v
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/r05i_prof_$v" -o run --output-format csv \
    -- tests/cpp/bin/dense_bench_$v 15 15 10 > gpurun_out/r05i_prof_$v.log 2>&1 || exit $?
  f=$(find gpurun_out/r05i_prof_$v -name '*kernel_stats.csv' | head -1)
  echo "== $v"; cut -c1-200 "$f"
done
