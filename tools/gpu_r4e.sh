#!/bin/bash
# Round 4: fused cost-volume backward without spills -- its tests and the flow bench, the fp32
# bench with it on and off.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=${1:-gpurun_out/r4e}
mkdir -p "$OUT"
run() {
  local t=$1; shift
  timeout -k 10 "$t" "$@"; local rc=$?
  case $rc in 124|134|137|139) echo "step '$*' rc $rc: stopping"; exit $rc;; esac
  return $rc
}
run 600 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_gpu_kernels.py \
  -k "cost_volume or corr_concat" > "$OUT/kern.log" 2>&1; echo "kernel tests rc $?"
grep -E "^(FAILED|ERROR)|passed|failed" "$OUT/kern.log" | tail -15
run 300 python tools/flow_bench.py --flow-scale 0.3 > "$OUT/flow_bench.txt" 2>&1; echo "flow bench rc $?"; grep -v amdgpu "$OUT/flow_bench.txt"
bash tools/gpu_ab.sh "$OUT/ab" 2 'fused|OFLOW_TUNE=9=5|--steps 20 --warmup 5' 'sep|OFLOW_TUNE=9=1|--steps 20 --warmup 5'
