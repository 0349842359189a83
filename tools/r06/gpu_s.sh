#!/bin/bash
# round 6, pass s: drhip_sort under skewed digit distributions (tools/r06/sort_skew_probe.py)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06s
timeout -k 10 400 python3 tools/r06/sort_skew_probe.py 2>&1 | tee gpurun_out/r06s/sort_skew_probe.txt
