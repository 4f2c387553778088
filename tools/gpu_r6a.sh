#!/bin/bash
# Round 6, first GPU call: the round-5 crash subset after the one-stream reducer fix, the
# restored kernel tests and the training-BN tests, then the torch-free C++ reproducer of the
# graph-replay fault (last: a fault ends the call).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=${1:-gpurun_out/r6a}
mkdir -p "$OUT"
run() {
  local t=$1; shift
  timeout -k 10 "$t" "$@"; local rc=$?
  case $rc in 124|134|137|139) echo "step '$*' rc $rc: stopping"; exit $rc;; esac
  return $rc
}
PT="python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider"
OFLOW_NATIVE_BT=1 run 300 $PT -p no:faulthandler tests/test_gpu_bn_train.py tests/test_gpu_dist.py tests/test_gpu_graph.py -k "mode_switch or world1 or steps_vs_oracle" > "$OUT/subset.log" 2>&1; echo "subset rc $?"; tail -3 "$OUT/subset.log"
run 900 $PT tests/test_gpu_kernels_misc.py tests/test_gpu_bn_train.py tests/test_gpu_dist.py tests/test_gpu_graph.py > "$OUT/tests.log" 2>&1; echo "tests rc $?"; grep -E "^FAILED|^ERROR|passed|failed" "$OUT/tests.log" | tail -12
