#!/bin/bash
# Round 4: conv_halo_b16's direct epilogue + act' sign masks -- kernel / module / config-3 tests,
# the per-layer bench, the bf16 B=32 step A/B (direct + masks vs the general epilogue).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=${1:-gpurun_out/r4f}
mkdir -p "$OUT"
run() {
  local t=$1; shift
  timeout -k 10 "$t" "$@"; local rc=$?
  case $rc in 124|134|137|139) echo "step '$*' rc $rc: stopping"; exit $rc;; esac
  return $rc
}
run 600 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_gpu_kernels.py \
  -k "b16i" > "$OUT/kern.log" 2>&1; echo "kernel tests rc $?"
grep -E "^(FAILED|ERROR)|passed|failed|Error" "$OUT/kern.log" | tail -15
run 900 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_gpu_bf16_modules.py \
  "tests/test_gpu_fullsize.py::test_config3_384x512_b32_bf16" "tests/test_gpu_graph.py" > "$OUT/tests.log" 2>&1; echo "tests rc $?"
grep -E "^(FAILED|ERROR)|passed|failed|worst" "$OUT/tests.log" | tail -30
run 300 python tools/b16i_bench.py --batch 32 --ablate > "$OUT/b16i_b32.txt" 2>&1; echo "b16i rc $?"; grep -v amdgpu.ids "$OUT/b16i_b32.txt" | head -8
bash tools/gpu_ab.sh "$OUT/ab" 2 'direct||--precision bf16 --batch 32 --steps 10 --warmup 3' \
  'general|OFLOW_B16I_MASK=0 OFLOW_TUNE=22=0|--precision bf16 --batch 32 --steps 10 --warmup 3'
