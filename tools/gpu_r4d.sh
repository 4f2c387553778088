#!/bin/bash
# Round 4: the b16i wgrad swizzle fix and the fused cost-volume backward -- kernel tests, the
# bf16 module / model / DP / config-3 tests, the flow and b16i microbenchmarks, both benches.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=${1:-gpurun_out/r4d}
mkdir -p "$OUT"
# A step that faulted, aborted, crashed or ran out of time ends the call (test failures do not).
run() {
  local t=$1; shift
  timeout -k 10 "$t" "$@"; local rc=$?
  case $rc in 124|134|137|139) echo "step '$*' rc $rc: stopping"; exit $rc;; esac
  return $rc
}
run 600 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_gpu_kernels.py \
  -k "b16i or cost_volume or corr_concat" > "$OUT/kern.log" 2>&1; echo "kernel tests rc $?"
grep -E "^(FAILED|ERROR)|passed|failed" "$OUT/kern.log" | tail -15
run 300 python tools/flow_bench.py --flow-scale 0.3 > "$OUT/flow_bench.txt" 2>&1; echo "flow bench rc $?"; grep -v amdgpu "$OUT/flow_bench.txt"
run 900 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_gpu_bf16_modules.py \
  "tests/test_gpu_model.py::test_bn_gamma_near_zero" "tests/test_gpu_dist.py" \
  "tests/test_gpu_fullsize.py::test_config3_384x512_b32_bf16" > "$OUT/tests.log" 2>&1; echo "tests rc $?"
grep -E "^(FAILED|ERROR)|passed|failed|median|worst" "$OUT/tests.log" | tail -30
run 300 python tools/b16i_bench.py --batch 32 --ablate > "$OUT/b16i_b32.txt" 2>&1; echo "b16i rc $?"; grep -v amdgpu.ids "$OUT/b16i_b32.txt" | tail -12
run 300 python bench.py --precision bf16 --batch 32 --no-cpu-baseline --steps 10 --warmup 3 > "$OUT/bench_bf16.log" 2>&1; echo "bench bf16 rc $?"
grep '^{' "$OUT/bench_bf16.log" | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'])"
run 600 python bench.py --steps 20 --warmup 5 > "$OUT/bench.log" 2>&1; echo "bench fp32 rc $?"; grep '^{' "$OUT/bench.log" | head -c 400; echo
