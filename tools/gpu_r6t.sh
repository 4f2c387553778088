#!/bin/bash
# multi-stream capture, replays on a high-priority stream: the round-5 crashing subset
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
OUT=${1:-gpurun_out/r6t}
mkdir -p "$OUT"
PT="python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider"
OFLOW_GRAPH_STREAMS=multi OFLOW_GRAPH_REPLAY_PRIO=-1 timeout -k 10 300 $PT tests/test_gpu_bn_train.py tests/test_gpu_dist.py tests/test_gpu_graph.py -k "mode_switch or world1 or steps_vs_oracle" > "$OUT/subset.log" 2>&1; r=$?
echo "subset rc $r"; grep -E "PASSED|FAILED|passed|failed" "$OUT/subset.log" | tail -12
exit $r
