#!/bin/bash
# round 6, pass c: the standalone reproducer (tools/pool_tlb_repro, no
# libdrhip) on pass a's allocation traces (tools/r06/traces), pool and
# hipMalloc; then the counter passes of tools/r06/pmc_limiters.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06c
mkdir -p $O
for t in A1 A3 A4; do
  for a in pool hipmalloc; do
    timeout -k 10 180 tools/pool_tlb_repro tools/r06/traces/trace_$t.txt --alloc $a --reps 3 > $O/repro_${t}_$a.txt 2>&1; rc=$?
    echo "repro $t $a rc $rc: $(tail -1 $O/repro_${t}_$a.txt) | $(grep -m3 WRONG $O/repro_${t}_$a.txt | tr '\n' ' ')"
    [ $rc -ge 124 ] && exit $rc
  done
done
bash tools/r06/pmc_limiters.sh
