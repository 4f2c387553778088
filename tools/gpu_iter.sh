#!/bin/bash
# Iteration loop on one GPU box: targeted GPU tests, then kernel micro-benchmarks, then the
# bench without the CPU baseline.  Usage: tools/gpu_iter.sh "<pytest -k expr>" [flow|conv|none]
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q -k "$1" > gpurun_out/pytest_iter.log 2>&1
st=$?
tail -5 gpurun_out/pytest_iter.log
[ $st -ne 0 ] && exit $st
if [ "$2" = "flow" ]; then
  timeout -k 10 300 python tools/flow_bench.py || exit $?
elif [ "$2" = "conv" ]; then
  timeout -k 10 300 python tools/conv_bench.py --reps 10 || exit $?
fi
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_iter.log 2>&1
st=$?
tail -3 gpurun_out/bench_iter.log | cut -c1-600
exit $st
