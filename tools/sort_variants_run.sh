#!/bin/bash
# time drhip_sort at 2^N u32 with libdrhip.so variants under tools/diag/<name>
# (built by VAR_ROOT=diag tools/build_variant.sh <name> sort "<flags>")
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
for v in base ${VARIANTS}; do
  if [ $v = base ]; then LP=$R/distributed-ranges_amd; else LP=$R/tools/diag/$v; fi
  for rep in 1 2; do
    env LD_LIBRARY_PATH=$LP timeout -k 10 60 ./tools/sort_bench ${LOG2N:-28} 5 > /tmp/sb.txt || exit $?
    echo "$v $(head -1 /tmp/sb.txt)"
  done
done
