#!/bin/bash
# tiled mode-A deterministic warp backward: bitwise tests, the det tests, timings both ways
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
OUT=${1:-gpurun_out/r6y}
mkdir -p "$OUT"
PT="python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 400 $PT tests/test_gpu_kernels_misc.py tests/test_gpu_kernels.py -k "warp" > $OUT/tests.log 2>&1; r=$?
echo "tests rc $r"; grep -E "^FAILED|passed|failed" $OUT/tests.log | tail -8
[ $r -eq 0 ] || exit $r
for k in 0 1 P; do
  T=34=$k; [ $k = P ] && T=34=1,35=1
  OFLOW_TUNE=$T timeout -k 10 200 python tools/flow_bench.py --flow-scale 0.3 > $OUT/flow_k$k.txt 2>&1; echo "flow k$k rc $?"
  grep -o "level . [^|]*|\|warp_bwd_det[^|]*|" $OUT/flow_k$k.txt | paste - - | head -4
done
for k in 0 1 P; do
  T=34=$k; [ $k = P ] && T=34=1,35=1
  OFLOW_TUNE=$T timeout -k 10 200 python tools/flow_bench.py --flow-scale 0.3 --batch 32 > $OUT/flow32_k$k.txt 2>&1; echo "flow32 k$k rc $?"
  grep -o "level . [^|]*|\|warp_bwd_det[^|]*|" $OUT/flow32_k$k.txt | paste - - | head -4
done
