#!/bin/bash
# GPU tests (pytest -k $1), then A/B: conv_bench on $2 layers and the whole-step bench, for the
# default library and every _build/ab_*/liboflow.so, interleaved ROUNDS ($3, default 2) times.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -n "$1" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$1" > gpurun_out/pytest_iter.log 2>&1
  st=$?; tail -3 gpurun_out/pytest_iter.log; [ $st -ne 0 ] && exit $st
fi
for i in $(seq ${3:-2}); do
  for d in base optical_flow_amd/_build/ab_*; do
    if [ "$d" = base ]; then lib=optical_flow_amd/liboflow.so; else lib=$d/liboflow.so; fi
    [ -f $lib ] || continue
    echo "== $(basename $d) round $i"
    if [ -n "$2" ]; then OFLOW_LIB=$lib timeout -k 10 120 python tools/conv_bench.py --reps 10 --only "$2" 2>&1 | grep -v amdgpu.ids || exit 1; fi
    OFLOW_LIB=$lib timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --timing-steps 0 2>/dev/null | grep '^{' | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench', d['value'], d['ms_per_step'])" || exit 1
  done
done
