#!/bin/bash
# Round 4: direct epilogue + masks -- module / config-3 / graph tests, per-layer bench with the
# mask_in input gradient, the bf16 B=32 bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=${1:-gpurun_out/r4g}
mkdir -p "$OUT"
run() {
  local t=$1; shift
  timeout -k 10 "$t" "$@"; local rc=$?
  case $rc in 124|134|137|139) echo "step '$*' rc $rc: stopping"; exit $rc;; esac
  return $rc
}
run 900 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_gpu_bf16_modules.py \
  "tests/test_gpu_fullsize.py::test_config3_384x512_b32_bf16" "tests/test_gpu_graph.py" \
  "tests/test_gpu_model.py::test_bn_gamma_near_zero" > "$OUT/tests.log" 2>&1; echo "tests rc $?"
grep -E "^(FAILED|ERROR)|passed|failed|worst|Error" "$OUT/tests.log" | tail -30
run 300 python tools/b16i_bench.py --batch 32 > "$OUT/b16i_b32.txt" 2>&1; echo "b16i rc $?"; grep -v amdgpu.ids "$OUT/b16i_b32.txt"
run 300 python bench.py --precision bf16 --batch 32 --no-cpu-baseline --steps 10 --warmup 3 > "$OUT/bench_bf16.log" 2>&1; echo "bench bf16 rc $?"
grep '^{' "$OUT/bench_bf16.log" | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac']); [print(k, v) for k, v in d['roofline']['per_kernel'].items()]"
