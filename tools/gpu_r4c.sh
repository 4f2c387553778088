#!/bin/bash
# Round 4: bf16-image kernels per layer (A/B vs the fp32-image halo kernels), the module tests
# on both paths, the BN guard / det-warp / graph / DP tests, the bf16 B=32 bench with and
# without images, the trajectory runs.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=${1:-gpurun_out/r4c}
mkdir -p "$OUT"
# A step that faulted, aborted, crashed or ran out of time ends the call (test failures do not).
run() {
  local t=$1; shift
  timeout -k 10 "$t" "$@"; local rc=$?
  case $rc in 124|134|137|139) echo "step '$*' rc $rc: stopping"; exit $rc;; esac
  return $rc
}
run 300 python tools/b16i_bench.py --batch 32 --ablate > "$OUT/b16i_b32.txt" 2>&1; echo "b16i b32 rc $?"; grep -v amdgpu.ids "$OUT/b16i_b32.txt" | tail -14
run 900 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_gpu_bf16_modules.py \
  "tests/test_gpu_model.py::test_bn_gamma_near_zero" "tests/test_gpu_model.py::test_resnet_block_bn_guard" \
  "tests/test_gpu_model.py::test_two_forwards_one_backward" "tests/test_gpu_model.py::test_flow_net_forward_backward" \
  "tests/test_gpu_kernels.py::test_warp_bwd_deterministic" \
  "tests/test_gpu_graph.py::test_graph_matches_eager" "tests/test_gpu_dist.py" "tests/test_gpu_fullsize.py::test_config3_384x512_b32_bf16" \
  > "$OUT/tests.log" 2>&1; echo "tests rc $?"
grep -E "worst|PASSED|FAILED|Error|grad rel_l2|replay" "$OUT/tests.log" | head -120
run 300 python bench.py --precision bf16 --batch 32 --no-cpu-baseline --steps 10 --warmup 3 > "$OUT/bench_bf16.log" 2>&1; echo "bench img rc $?"
grep '^{' "$OUT/bench_bf16.log" | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac']); [print(k, v) for k, v in d['roofline']['per_kernel'].items()]"
OFLOW_B16I=0 run 300 python bench.py --precision bf16 --batch 32 --no-cpu-baseline --steps 10 --warmup 3 > "$OUT/bench_bf16_off.log" 2>&1; echo "bench off rc $?"
grep '^{' "$OUT/bench_bf16_off.log" | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'])"
run 300 python tools/flow_bench.py --flow-scale 0.3 > "$OUT/flow_bench.txt" 2>&1; echo "flow bench rc $?"; cat "$OUT/flow_bench.txt" | grep -v amdgpu
run 600 python tools/hip_trajectory.py --steps 26 --det --oracle-every 5 --out "$OUT/traj_det.jsonl" > "$OUT/traj_det.log" 2>&1; echo "traj det rc $?"
run 300 python tools/hip_trajectory.py --steps 26 --out "$OUT/traj_atomic.jsonl" > "$OUT/traj_atomic.log" 2>&1; echo "traj atomic rc $?"
run 600 python bench.py --steps 20 --warmup 5 > "$OUT/bench.log" 2>&1; echo "bench fp32 rc $?"; grep '^{' "$OUT/bench.log" | head -c 600; echo
