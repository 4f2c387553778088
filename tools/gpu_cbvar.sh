#!/bin/bash
# conv_bench on layers $1 for the base library and every _build/ab_* variant ($2 rounds)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
for i in $(seq ${2:-1}); do
for d in base optical_flow_amd/_build/ab_*; do
  if [ "$d" = base ]; then lib=optical_flow_amd/liboflow.so; else lib=$d/liboflow.so; fi
  echo "== $(basename $d)"
  OFLOW_LIB=$lib timeout -k 10 120 python tools/conv_bench.py --reps 10 --only "$1" 2>&1 | grep -v amdgpu.ids || exit 1
done
done
