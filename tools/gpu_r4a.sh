#!/bin/bash
# Round 4, first GPU call: the deterministic warp backward (kernel, graph and RCCL tests), the
# BN gamma guard, the flow micro-bench with the det form, the HIP training trajectory from the
# bench start (det, and the atomic default) and one default bench line.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=${1:-gpurun_out/r4a}
mkdir -p "$OUT"
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; }
run 300 python tools/b16i_bench.py --batch 8 > "$OUT/b16i_b8.txt" 2>&1; echo "b16i b8 rc $?"; cat "$OUT/b16i_b8.txt"
run 300 python tools/b16i_bench.py --batch 32 > "$OUT/b16i_b32.txt" 2>&1; echo "b16i b32 rc $?"; cat "$OUT/b16i_b32.txt"
run 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  "tests/test_gpu_kernels.py::test_warp_bwd_deterministic" \
  "tests/test_gpu_kernels.py::test_warp" "tests/test_gpu_kernels.py::test_warp_bwd_forms" \
  "tests/test_gpu_model.py::test_bn_gamma_near_zero" \
  "tests/test_gpu_model.py::test_flow_net_forward_backward" \
  "tests/test_gpu_graph.py::test_graph_matches_eager" \
  "tests/test_gpu_dist.py::test_rccl_dp_step_world1" > "$OUT/pytest.log" 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" "$OUT/pytest.log" | tail -40
[ $rc -eq 0 ] || { echo "tests rc $rc"; exit 1; }
run 300 python tools/flow_bench.py --flow-scale 0.3 > "$OUT/flow_bench.txt" 2>&1 || { echo flow bench failed; tail -5 "$OUT/flow_bench.txt"; exit 1; }
run 300 python tools/flow_bench.py --flow-scale 0.3 --flow-offset 40 > "$OUT/flow_bench_off40.txt" 2>&1 || { echo flow bench 2 failed; exit 1; }
cat "$OUT/flow_bench.txt" "$OUT/flow_bench_off40.txt"
run 600 python tools/hip_trajectory.py --steps 26 --det --oracle-every 5 --out "$OUT/traj_det.jsonl" > "$OUT/traj_det.log" 2>&1 || { echo traj det failed; tail -5 "$OUT/traj_det.log"; exit 1; }
run 300 python tools/hip_trajectory.py --steps 26 --det --out "$OUT/traj_det2.jsonl" > "$OUT/traj_det2.log" 2>&1 || { echo traj det2 failed; exit 1; }
run 300 python tools/hip_trajectory.py --steps 26 --out "$OUT/traj_atomic.jsonl" > "$OUT/traj_atomic.log" 2>&1 || { echo traj atomic failed; exit 1; }
cmp "$OUT/traj_det.jsonl" "$OUT/traj_det2.jsonl" > /dev/null && echo "det trajectories: identical files" || echo "det trajectories differ (oracle fields in run 1)"
run 600 python bench.py --steps 20 --warmup 5 > "$OUT/bench.log" 2>&1 || { echo bench failed; tail -5 "$OUT/bench.log"; exit 1; }
grep '^{' "$OUT/bench.log" | head -c 400; echo
run 600 python bench.py --steps 20 --warmup 5 --deterministic 1 --no-cpu-baseline > "$OUT/bench_det.log" 2>&1 || { echo bench det failed; tail -5 "$OUT/bench_det.log"; exit 1; }
grep '^{' "$OUT/bench_det.log" | head -c 300; echo
echo done
