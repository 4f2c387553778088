#!/bin/bash
# Round 4: bf16-image kernels per layer (A/B vs the fp32-image halo kernels), the module tests
# on both paths, the BN guard tests, and the bf16 B=32 bench with / without images.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=${1:-gpurun_out/r4c}
mkdir -p "$OUT"
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; }
run 300 python tools/b16i_bench.py --batch 32 > "$OUT/b16i_b32.txt" 2>&1; echo "b16i b32 rc $?"; grep -v amdgpu.ids "$OUT/b16i_b32.txt" | tail -14
run 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_bf16_modules.py \
  "tests/test_gpu_model.py::test_bn_gamma_near_zero" "tests/test_gpu_model.py::test_resnet_block_bn_guard" \
  > "$OUT/tests.log" 2>&1; echo "tests rc $?"
grep -E "worst|PASSED|FAILED|Error|rel_l2 [0-9.e+-]+$" "$OUT/tests.log" | grep -v "rel_l2 [0-9].[0-9][0-9]e-0[5-9]" | head -70
run 300 python bench.py --precision bf16 --batch 32 --no-cpu-baseline --steps 10 --warmup 3 > "$OUT/bench_bf16.log" 2>&1; echo "bench img rc $?"
grep '^{' "$OUT/bench_bf16.log" | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac']); [print(k, v) for k, v in d['roofline']['per_kernel'].items()]"
OFLOW_B16I=0 run 300 python bench.py --precision bf16 --batch 32 --no-cpu-baseline --steps 10 --warmup 3 > "$OUT/bench_bf16_off.log" 2>&1; echo "bench off rc $?"
grep '^{' "$OUT/bench_bf16_off.log" | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'])"
