#!/bin/bash
# flow_bench over every _build/ab_* variant and the base library at flow scale $1 (default 0.3)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
for d in base optical_flow_amd/_build/ab_*; do
  if [ "$d" = base ]; then lib=optical_flow_amd/liboflow.so; else lib=$d/liboflow.so; fi
  echo "== $(basename $d)"
  OFLOW_LIB=$lib timeout -k 10 120 python tools/flow_bench.py --reps 10 --flow-scale ${1:-0.3} 2>&1 | grep -v amdgpu.ids || exit 1
done
