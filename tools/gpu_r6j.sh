#!/bin/bash
# graph-replay fault: the crashing subset with a native backtrace (tools/crash_bt.c; -s so that
# pytest's fd capture does not swallow it).  A 1 GiB main-thread stack did not avoid the fault
# (gpurun_out/r6j/bigstack.log): not a stack overflow.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
OUT=${1:-gpurun_out/r6k}
mkdir -p "$OUT"
PT="python -u -m pytest -v -s --timeout 300 --timeout-method thread -p no:cacheprovider -p no:faulthandler"
OFLOW_NATIVE_BT=1 timeout -k 10 300 $PT tests/test_gpu_bn_train.py tests/test_gpu_dist.py tests/test_gpu_graph.py -k "mode_switch or world1 or steps_vs_oracle" > "$OUT/defstack.log" 2>&1; r=$?
echo "default stack rc $r"; grep crash_bt "$OUT/defstack.log" | head -70
exit $r
