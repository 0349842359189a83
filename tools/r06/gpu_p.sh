#!/bin/bash
# round 6, pass p: the standalone pool reproducer (tools/pool_tlb_repro, no
# libdrhip) again on a fresh box, now also with the blocks filled by a KERNEL
# instead of the copy engine (--fill kernel): which engine's writes go astray.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06p2
mkdir -p $O
for t in A1 A3; do
  for cfg in "pool copy" "pool kernel" "hipmalloc copy" "hipmalloc kernel"; do
    set -- $cfg
    timeout -k 10 180 tools/pool_tlb_repro tools/r06/traces/trace_$t.txt --alloc $1 --fill $2 --reps 3 > $O/repro_${t}_$1_$2.txt 2>&1; rc=$?
    echo "trace $t $1 $2 rc $rc: $(tail -1 $O/repro_${t}_$1_$2.txt)"
    [ $rc -ge 124 ] && exit $rc
  done
done
exit 0
