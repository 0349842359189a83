#!/bin/bash
# XCD-grouped onesweep: group-size sweep at 2^28 and 2^26 u32
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for g in 8 16 32 64 128 256; do
  echo "== group $g"
  DRHIP_SORT_OS_PT=1 DRHIP_SORT_OS_GROUP=$g timeout -k 10 60 ./tools/sort_bench 28 5 | grep drhip || exit 1
  DRHIP_SORT_OS_PT=1 DRHIP_SORT_OS_GROUP=$g timeout -k 10 60 ./tools/sort_bench 26 5 | grep drhip || exit 1
done
echo "== one-shot"
DRHIP_SORT_OS_PT=0 timeout -k 10 60 ./tools/sort_bench 26 5 | grep drhip
