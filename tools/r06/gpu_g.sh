#!/bin/bash
# round 6, pass g: (1) the dot kernel in three contexts on ONE box -- the
# round-5 A/B tool (fresh process, back-to-back launches), the bench's dot op
# alone, and the dot op at its place in the full bench; (2) FETCH_SIZE /
# WRITE_SIZE over every op of the default bench at HEAD (two separate PMC
# passes), the int64 gemv ops included.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R=$(pwd)
export TMPDIR=/tmp
O=gpurun_out/r06g
mkdir -p $O
for rep in 1 2; do
  echo "rep $rep ab_tool $(timeout -k 10 300 python3 tools/archive/r05/dot_ab.py base=distributed-ranges_amd/libdrhip.so | tail -1)" || exit 1
  timeout -k 10 300 python3 bench.py --only-ops dot --log2n 24 --steps 20 --warmup 3 --no-cpu-baseline > $O/dot_alone_$rep.json 2> $O/dot_alone_$rep.err || exit 1
  python3 -c "
import json; o=json.load(open('$O/dot_alone_$rep.json'))['ops']['dot']
print('rep $rep dot_alone kernel %.4f loop %.4f frac %.3f loop_frac %.3f' % (o['kernel_ms'], o['loop_kernel_ms'], o['frac'], o['loop_frac']))"
  timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_full_$rep.json 2> $O/bench_full_$rep.err || exit 1
  python3 -c "
import json; o=json.load(open('$O/bench_full_$rep.json'))['ops']['dot']
print('rep $rep dot_in_bench kernel %.4f loop %.4f frac %.3f loop_frac %.3f' % (o['kernel_ms'], o['loop_kernel_ms'], o['frac'], o['loop_frac']))"
done
rm -rf $O/pmc_fetch $O/pmc_write
timeout -s KILL 500 rocprofv3 --pmc FETCH_SIZE -d "$R/$O/pmc_fetch" -o pmc --output-format csv \
  -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline > $O/pmc_fetch.log 2>&1 || exit $?
echo "fetch pass done"
timeout -s KILL 500 rocprofv3 --pmc WRITE_SIZE -d "$R/$O/pmc_write" -o pmc --output-format csv \
  -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline > $O/pmc_write.log 2>&1 || exit $?
echo "write pass done"
python3 tools/pmc_summary.py $O/pmc_fetch $O/pmc_write > $O/r06_pmc_summary_all_ops.json
python3 - <<PY
import json
d = json.load(open("$O/r06_pmc_summary_all_ops.json"))
for k, v in d["kernels"].items():
    if k.startswith("void drhip") or "drhip::" in k:
        print(k[:80], {a: b for a, b in v.items() if "bytes" in a or "launches" in a})
PY
