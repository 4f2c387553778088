#!/bin/bash
# correlation lanes-per-pixel A/B (of_set_tuning key 9): GPU corr tests per form, flow_bench, step bench
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
for t in "9=8" "9=4"; do
  OFLOW_TUNE=$t timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests -k "corr or cost or flow_module or model" > gpurun_out/pytest_corr.log 2>&1 || { tail -30 gpurun_out/pytest_corr.log; exit 1; }
  echo "tests $t: $(tail -1 gpurun_out/pytest_corr.log)"
done
for i in 1 2; do for t in "9=8" "9=4"; do echo "flow_bench $t"; OFLOW_TUNE=$t timeout -k 10 120 python tools/flow_bench.py --reps 10 2>&1 | grep -v amdgpu.ids | sed 's/| warp_fwd.*//' || exit 1; done; done
bash tools/gpu_abenv.sh 2 "lpp4:OFLOW_TUNE=9=4"
