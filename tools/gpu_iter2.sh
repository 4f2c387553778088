#!/bin/bash
# GPU iteration: targeted GPU tests (pytest -k expr), then conv micro-bench on the given layers,
# then the default bench.   tools/gpu_iter2.sh "<pytest -k expr>" "<conv layers or ''>"
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$1" > gpurun_out/pytest_iter.log 2>&1
st=$?; tail -5 gpurun_out/pytest_iter.log; [ $st -ne 0 ] && exit $st
if [ -n "$2" ]; then timeout -k 10 300 python tools/conv_bench.py --reps 10 --only "$2" 2>&1 | grep -v amdgpu.ids || exit 1; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_iter.log 2>&1
st=$?; grep '^{' gpurun_out/bench_iter.log | cut -c1-330; exit $st
