#!/bin/bash
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q -rA > gpurun_out/pytest_gpu.log 2>&1
st=$?
echo "pytest exit $st"
tail -40 gpurun_out/pytest_gpu.log
if [ $st -ne 0 ] && [ $st -ne 1 ]; then exit $st; fi
timeout -k 10 600 python bench.py --steps 5 --warmup 2 --cpu-steps 1 > gpurun_out/bench1.log 2>&1
st=$?
echo "bench exit $st"
tail -5 gpurun_out/bench1.log
exit $st
