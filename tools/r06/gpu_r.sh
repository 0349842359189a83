#!/bin/bash
# round 6, pass r: drhip_sort per key type at 1 GiB of keys (tools/r06/sort64_probe.py)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06r
timeout -k 10 300 python3 tools/r06/sort64_probe.py 2>&1 | tee gpurun_out/r06r/sort64_probe.txt
