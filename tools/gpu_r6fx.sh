#!/bin/bash
# fixed-point fallback grids of the deterministic warp backward (of_set_tuning key 37)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
OUT=${1:-gpurun_out/r6fx}
mkdir -p "$OUT"
PT="python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider"
OFLOW_TUNE=37=1 timeout -k 10 400 $PT tests/test_gpu_kernels.py tests/test_gpu_kernels_misc.py -k "warp_bwd_det" > $OUT/tests.log 2>&1; r=$?
echo "tests rc $r"; grep -E "^FAILED|passed|failed" $OUT/tests.log | tail -5
[ $r -eq 0 ] || exit $r
for k in 0 1 2 4 0 1; do
  OFLOW_TUNE=37=$k timeout -k 10 200 python tools/flow_bench.py --flow-scale 0.3 > $OUT/flow_k$k.txt 2>&1 || { echo "flow k$k failed"; exit 1; }
  echo "k$k"; grep -o "level . [^|]*|\|warp_bwd_det[^|]*|" $OUT/flow_k$k.txt | paste - - | head -3
done
