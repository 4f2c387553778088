#!/bin/bash
# Round 4: the direct epilogue for fp32 outputs too -- kernel / module / config-3 tests,
# per-layer bench, bf16 B=32 bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=${1:-gpurun_out/r4k}
mkdir -p "$OUT"
run() {
  local t=$1; shift
  timeout -k 10 "$t" "$@"; local rc=$?
  case $rc in 124|134|137|139) echo "step '$*' rc $rc: stopping"; exit $rc;; esac
  return $rc
}
run 600 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_gpu_kernels.py \
  -k "b16i" tests/test_gpu_bf16_modules.py "tests/test_gpu_fullsize.py::test_config3_384x512_b32_bf16" \
  > "$OUT/tests.log" 2>&1; echo "tests rc $?"
grep -E "^(FAILED|ERROR)|passed|failed|Error" "$OUT/tests.log" | tail -15
run 300 python tools/b16i_bench.py --batch 32 > "$OUT/b16i_b32.txt" 2>&1; echo "b16i rc $?"; grep -v amdgpu.ids "$OUT/b16i_b32.txt" | head -12
A='--precision bf16 --batch 32 --steps 10 --warmup 3'
bash tools/gpu_ab.sh "$OUT/ab" 2 "direct||$A" "nodirect32|OFLOW_TUNE=22=0|$A"
