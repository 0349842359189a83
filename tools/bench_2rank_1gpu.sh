#!/bin/bash
# Rehearse bench.py's N=2 code path on a 1-GPU box: two ranks (NPROC=n for
# more) on the same device (LOCAL_RANK forced to 0).  Small sizes; correctness of the RCCL
# path only, the numbers mean nothing.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
# two processes on ONE device: no persistent (resident-grid) sort, whose
# grids from separate processes could starve each other (drhip.h sort note)
export DRHIP_FORCE_LOCAL0=1 DRHIP_BENCH_BACKEND=gloo DRHIP_SORT_OS_PT=0
NP=${NPROC:-2}
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $NP --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus $NP --steps 3 --warmup 1 --log2n 24 --sort-log2n ${SORT_LOG2N:-22} --gemv-log2m 22 \
  --stencil-log2n 22 --no-cpu-baseline
