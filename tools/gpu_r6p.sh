#!/bin/bash
# eager side streams on/off: the training-BN whole-step test and the det graph-vs-eager test
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
OUT=${1:-gpurun_out/r6p}
mkdir -p "$OUT"
PT="python -u -m pytest -v -s --timeout 300 --timeout-method thread -p no:cacheprovider"
T="tests/test_gpu_bn_train.py::test_flow_net_bn_training tests/test_gpu_graph.py::test_graph_matches_eager"
timeout -k 10 300 $PT $T -k "fp32" > "$OUT/side_on.log" 2>&1; echo "side on rc $?"
OFLOW_SIDE_MAX_PIX=0 OFLOW_BN_SIDE=0 OFLOW_PROJ_SIDE=0 timeout -k 10 300 $PT $T -k "fp32" > "$OUT/side_off.log" 2>&1; echo "side off rc $?"
OFLOW_BN_SIDE=0 timeout -k 10 300 $PT $T -k "fp32" > "$OUT/bnside_off.log" 2>&1; echo "bn side off rc $?"
for f in side_on side_off bnside_off; do echo "== $f"; grep -E "fp32: flows|replay|PASSED|FAILED" "$OUT/$f.log" | head -20; done
