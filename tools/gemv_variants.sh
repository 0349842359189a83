cd "${GRAFT_REPO_ROOT:-/root/repo}"
for v in base nt nty ntboth base; do
  if [ $v = base ]; then unset DRHIP_LIB; else export DRHIP_LIB=$PWD/tools/var/$v/libdrhip.so; fi
  timeout -k 10 120 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --only-ops gemv --log2n 24 > gpurun_out/gv_$v.log 2>&1 || exit 1
  python -c "
import json,sys
d=json.loads([l for l in open('gpurun_out/gv_$v.log') if l.startswith('{')][-1])
print('$v', 'banded', round(d['ops']['gemv_banded']['kernel_ms'],4), round(d['ops']['gemv_banded']['frac'],4), 'random', round(d['ops']['gemv']['kernel_ms'],3))"
done
