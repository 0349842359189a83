#!/bin/bash
# onesweep sub-tile sweep (tools/var/kplNN built by tools/build_variant.sh) at 2^28 u32
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
mkdir -p gpurun_out
for v in base ${VARIANTS:-kpl24 kpl40 kpl48}; do
  if [ $v = base ]; then LP=$R/distributed-ranges_amd; else LP=$R/tools/var/$v; fi
  for rep in 1 2; do
    env LD_LIBRARY_PATH=$LP DRHIP_SORT_ALGO=onesweep timeout -k 10 60 ./tools/sort_bench 28 5 > gpurun_out/sb.txt || exit $?
    echo "$v $(head -1 gpurun_out/sb.txt)"
  done
done
