#!/bin/bash
# round 6: counter passes naming the limiter of the banded C4 SpMV
# (spmv_csr_stream_kernel) and of the sort's look-back passes
# (radix_onesweep_pt passes 1-3 vs pass 0), one rocprofv3 --pmc pass per
# counter group over the same short bench run; summary per kernel by
# tools/r06/pmc_kernels.py.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
export TMPDIR=/tmp
O=gpurun_out/r06pmc
rm -rf $O; mkdir -p $O
timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
ARGS="--only-ops ${OPS:-gemv_banded,sort} --log2n 24 --steps 3 --warmup 1 --no-cpu-baseline"
i=0
for group in \
  "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" \
  "SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_WAVES" \
  "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --pmc $group -d "$R/$O/p$i" -o pmc --output-format csv \
    -- python3 "$R/bench.py" $ARGS > $O/p$i.log 2>&1; rc=$?
  echo "pass $i rc $rc: $group"
  [ $rc -ne 0 ] && { tail -5 $O/p$i.log; [ $rc -ge 124 ] && exit $rc; }
done
python3 tools/r06/pmc_kernels.py $O/p1 $O/p2 $O/p3 > $O/summary.json
python3 -c "import json; d=json.load(open('$O/summary.json')); [print(k[:60], {c: round(v) for c, v in d[k].items()}) for k in d if 'spmv' in k or 'onesweep' in k or 'radix' in k]"
exit 0
