cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for m in default pinned; do timeout -k 10 120 python tools/dbg_fill.py $m || exit $?; done
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
bash tools/sort_stamps.sh || exit $?
bash tools/pmc_calib.sh
