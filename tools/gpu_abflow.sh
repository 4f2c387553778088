#!/bin/bash
# Flow-kernel A/B: GPU tests (-k $1) on every variant, then flow_bench base vs variants, and
# the whole-step bench, $2 rounds interleaved.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
for d in base optical_flow_amd/_build/ab_*; do
  if [ "$d" = base ]; then lib=optical_flow_amd/liboflow.so; else lib=$d/liboflow.so; fi
  OFLOW_LIB=$lib timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$1" > gpurun_out/pytest_$(basename $d).log 2>&1
  st=$?; echo "$(basename $d): $(tail -1 gpurun_out/pytest_$(basename $d).log)"; [ $st -ne 0 ] && { tail -30 gpurun_out/pytest_$(basename $d).log; exit $st; }
done
for i in $(seq ${2:-2}); do
  for d in base optical_flow_amd/_build/ab_*; do
    if [ "$d" = base ]; then lib=optical_flow_amd/liboflow.so; else lib=$d/liboflow.so; fi
    echo "== $(basename $d) round $i"
    OFLOW_LIB=$lib timeout -k 10 120 python tools/flow_bench.py --reps 10 2>&1 | grep -v amdgpu.ids || exit 1
    OFLOW_LIB=$lib timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --timing-steps 0 2>/dev/null | grep '^{' | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench', d['value'], d['ms_per_step'])" || exit 1
  done
done
