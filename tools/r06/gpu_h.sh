#!/bin/bash
# round 6, pass h: is the dot kernel's 3 % in-bench slowdown the GPU's state
# after the bench's earlier ops, or the placement of the bench's tensors?
# The A/B tool (fresh process) on a cool GPU, then right after a full bench;
# and the bench's dot op alone right after a full bench.  Then the C++
# one-process bench with the general-comparator sort.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06h
mkdir -p $O
dotab() { timeout -k 10 300 python3 tools/archive/r05/dot_ab.py base=distributed-ranges_amd/libdrhip.so | tail -1; }
echo "cool ab_tool: $(dotab)" || exit 1
for rep in 1 2; do
  timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_full_$rep.json 2> $O/bench_full_$rep.err || exit 1
  echo "rep $rep after-bench ab_tool: $(dotab)" || exit 1
  timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_full_b$rep.json 2> $O/bench_full_b$rep.err || exit 1
  timeout -k 10 300 python3 bench.py --only-ops dot --log2n 24 --steps 20 --warmup 20 --no-cpu-baseline > $O/dot_after_$rep.json 2> $O/dot_after_$rep.err || exit 1
  python3 -c "
import json
a=json.load(open('$O/bench_full_$rep.json'))['ops']['dot']; b=json.load(open('$O/dot_after_$rep.json'))['ops']['dot']
print('rep $rep in-bench kernel %.4f loop %.4f | dot alone right after a bench: kernel %.4f loop %.4f' % (a['kernel_ms'], a['loop_kernel_ms'], b['kernel_ms'], b['loop_kernel_ms']))"
done
echo "cool-down 60 s"; sleep 60
echo "after 60 s idle ab_tool: $(dotab)"
timeout -k 10 300 tests/cpp/bin/shp_bench --devices 0 --reps 5 > $O/shp_bench.json 2>&1; echo "shp_bench rc $?"; tail -c 1500 $O/shp_bench.json
