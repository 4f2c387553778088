#!/bin/bash
# warp backward forms (of_set_tuning key 7): GPU tests, flow_bench per form and flow spread,
# then the whole-step A/B ($1 rounds).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "warp" > gpurun_out/pytest_warp.log 2>&1 || { tail -30 gpurun_out/pytest_warp.log; exit 1; }
tail -2 gpurun_out/pytest_warp.log
for fs in 0.3 2.0; do
  for k in 1 0; do
    echo "flow-scale $fs key7=$k"
    OFLOW_TUNE=7=$k timeout -k 10 120 python tools/flow_bench.py --reps 10 --flow-scale $fs 2>/dev/null | grep -o "level [0-9].*warp_bwd *[0-9.]* us" | sed 's/| corr_fwd.*warp_bwd/ warp_bwd/' || exit 1
  done
done
bash tools/gpu_abenv.sh ${1:-2} "agg:OFLOW_TUNE=7=0"
