#!/bin/bash
# own_tile with d(flow)'s taps formed first: bitwise tests, flow timings (this build only)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
OUT=${1:-gpurun_out/r6tt}
mkdir -p "$OUT"
PT="python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 400 $PT tests/test_gpu_kernels_misc.py tests/test_gpu_kernels.py -k "warp_bwd_det" > $OUT/tests.log 2>&1; r=$?
echo "tests rc $r"; grep -E "^FAILED|^E  |passed|failed" $OUT/tests.log | head -8
[ $r -eq 0 ] || exit $r
for k in 1 2 1 2; do
  OFLOW_TUNE=34=$k timeout -k 10 200 python tools/flow_bench.py --flow-scale 0.3 > $OUT/flow_k$k.txt 2>&1 || { echo "flow k$k failed"; exit 1; }
  echo "k$k"; grep -o "level . [^|]*|\|warp_bwd_det[^|]*|" $OUT/flow_k$k.txt | paste - - | head -3
done
