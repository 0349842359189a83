cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_scan.py -m gpu -v --timeout 200 --timeout-method thread --durations=15 > gpurun_out/cfg.log 2>&1
rc=$?; tail -40 gpurun_out/cfg.log; exit $rc
