#!/bin/bash
# graph-replay fault: the crashing subset with HIP's graph executor on the launch stream only
# (DEBUG_HIP_FORCE_GRAPH_QUEUES=1; the native backtrace put the fault in hip_graph_internal.cpp's
# parallel-stream assignment at launch, gpurun_out/r6k/defstack.log).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
OUT=${1:-gpurun_out/r6l}
mkdir -p "$OUT"
PT="python -u -m pytest -v -s --timeout 300 --timeout-method thread -p no:cacheprovider -p no:faulthandler"
DEBUG_HIP_FORCE_GRAPH_QUEUES=1 OFLOW_NATIVE_BT=1 timeout -k 10 300 $PT tests/test_gpu_bn_train.py tests/test_gpu_dist.py tests/test_gpu_graph.py -k "mode_switch or world1 or steps_vs_oracle" > "$OUT/q1.log" 2>&1; r=$?
echo "graph queues 1: rc $r"; grep -E "PASSED|FAILED|crash_bt\] #0[0-6]" "$OUT/q1.log" | head -20
exit $r
