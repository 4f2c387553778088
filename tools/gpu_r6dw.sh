#!/bin/bash
# deferred weight gradients of the large flow heads (OFLOW_DEFER_WGRAD): parity, A/B
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
OUT=${1:-gpurun_out/r6dw}
mkdir -p "$OUT"
PT="python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider"
OFLOW_DEFER_WGRAD=1 timeout -k 10 600 $PT tests/test_gpu_fullsize.py tests/test_gpu_model.py -k "config2 or flow_net or golden" > $OUT/tests.log 2>&1; r=$?
echo "tests rc $r"; grep -E "^FAILED|^E  |passed|failed" $OUT/tests.log | head -8
[ $r -eq 0 ] || exit $r
for rnd in 1 2 3; do
  for k in 1 0; do
    OFLOW_DEFER_WGRAD=$k timeout -k 10 300 python bench.py --no-cpu-baseline $BENCH_ARGS > $OUT/bench_k${k}_$rnd.log 2>&1 || { echo "bench k$k failed"; tail -3 $OUT/bench_k${k}_$rnd.log; exit 1; }
    echo "defer=$k $(grep -o '"value": [0-9.]*' $OUT/bench_k${k}_$rnd.log | head -1) $(grep -o '"final_loss": [0-9.]*' $OUT/bench_k${k}_$rnd.log | head -1)"
  done
done
