#!/bin/bash
# Correctness of every _build/ab_* variant (pytest -k $1 on it), then A/B: conv_bench on $2
# layers + the whole-step bench, base vs variants, $3 rounds interleaved.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
for d in optical_flow_amd/_build/ab_*; do
  [ -f $d/liboflow.so ] || continue
  OFLOW_LIB=$d/liboflow.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$1" > gpurun_out/pytest_$(basename $d).log 2>&1
  st=$?; echo "$(basename $d): $(tail -1 gpurun_out/pytest_$(basename $d).log)"; [ $st -ne 0 ] && { tail -30 gpurun_out/pytest_$(basename $d).log; exit $st; }
done
bash tools/gpu_ab2.sh "" "$2" ${3:-2}
