#!/bin/bash
# round 6, pass f: onesweep with every digit position counted in the
# pre-pass (DRHIP_SORT_H0_ALL=1, tools/var6/h0all) vs the default (passes 1-2
# count the next position under their write-out): sort parity with the
# variant, then three interleaved rounds of the bench's sort op (2^28 u32).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06f
mkdir -p $O
DRHIP_LIB=$PWD/tools/var6/h0all/libdrhip.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 \
  --timeout-method thread tests/test_gpu_sort.py -m gpu > $O/h0all_pytest.txt 2>&1; rc=$?
echo "h0all parity rc $rc: $(tail -1 $O/h0all_pytest.txt)"
[ $rc -ne 0 ] && { grep -E "FAILED|Error" $O/h0all_pytest.txt | tail -10; exit $rc; }
for rep in 1 2 3; do
  for v in base h0all; do
    if [ $v = base ]; then L=$PWD/distributed-ranges_amd/libdrhip.so; else L=$PWD/tools/var6/$v/libdrhip.so; fi
    DRHIP_LIB=$L timeout -k 10 300 python3 bench.py --only-ops sort --log2n 24 --steps 10 --warmup 2 --no-cpu-baseline \
      > $O/bench_${v}_$rep.json 2> $O/bench_${v}_$rep.err; rc=$?
    [ $rc -ne 0 ] && { tail -5 $O/bench_${v}_$rep.err; exit $rc; }
    python3 -c "
import json; d=json.load(open('$O/bench_${v}_$rep.json'))['ops']['sort']
print('rep $rep $v', round(d['local_sort_ms'], 4), round(d['frac'], 3), d['check']['ok'])"
  done
done
DRHIP_LIB=$PWD/tools/var6/h0all/libdrhip.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_h0all -o sort \
  --output-format csv -- python3 bench.py --only-ops sort --log2n 24 --steps 10 --warmup 2 --no-cpu-baseline > $O/prof_h0all.log 2>&1
echo "rocprof h0all rc $?"
