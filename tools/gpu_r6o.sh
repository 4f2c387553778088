#!/bin/bash
# single-stream graph capture: the round-5 crashing subset, then every graph / dist / BN-train /
# restored kernel test
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
OUT=${1:-gpurun_out/r6o}
mkdir -p "$OUT"
PT="python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider"
run() {
  local t=$1; shift
  timeout -k 10 "$t" "$@"; local rc=$?
  case $rc in 124|134|137|139) echo "step rc $rc: stopping"; exit $rc;; esac
  return $rc
}
run 300 $PT tests/test_gpu_bn_train.py tests/test_gpu_dist.py tests/test_gpu_graph.py -k "mode_switch or world1 or steps_vs_oracle" > "$OUT/subset.log" 2>&1; echo "subset rc $?"; grep -E "passed|failed" "$OUT/subset.log" | tail -2
run 900 $PT tests/test_gpu_kernels_misc.py tests/test_gpu_bn_train.py tests/test_gpu_dist.py tests/test_gpu_graph.py > "$OUT/tests.log" 2>&1; echo "tests rc $?"; grep -E "^FAILED|^ERROR|passed|failed" "$OUT/tests.log" | tail -12
