#!/bin/bash
# Onesweep per-tile phase breakdown: tools/sort_stamps against a stamped
# libdrhip.so variant, built on the CPU side with
#   VAR_ROOT=diag tools/build_variant.sh stamps sort -DDRHIP_SORT_STAMPS
# (tools/diag travels to the GPU box, tools/var does not).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for v in ${VARIANTS:-stamps}; do
  echo "== $v"
  LD_LIBRARY_PATH=$PWD/tools/diag/$v timeout -k 10 60 ./tools/sort_stamps ${LOG2N:-28} || exit $?
done
