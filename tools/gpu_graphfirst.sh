#!/bin/bash
# graph replays: high-priority stream for each capture's first launch only (REPLAY_FIRST_ONLY)
# -- the subset that crashed before the round-6 fix, the graph tests, then eager / graph benches
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
OUT=${1:-gpurun_out/r6gfirst}
mkdir -p "$OUT"
PT="python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $PT tests/test_gpu_bn_train.py tests/test_gpu_dist.py tests/test_gpu_graph.py -k "mode_switch or world1 or steps_vs_oracle" > $OUT/subset.log 2>&1; r=$?
echo "subset rc $r"; grep -E "^FAILED|Segmentation|passed|failed" $OUT/subset.log | head -5
[ $r -eq 0 ] || exit $r
timeout -k 10 600 $PT tests/test_gpu_graph.py tests/test_gpu_dist.py > $OUT/graph.log 2>&1; r=$?
echo "graph rc $r"; grep -E "^FAILED|Segmentation|passed|failed" $OUT/graph.log | head -5
[ $r -eq 0 ] || exit $r
for rnd in 1 2; do
  for gph in 0 1; do
    timeout -k 10 300 python bench.py --no-cpu-baseline --graph $gph > $OUT/bench_g${gph}_$rnd.log 2>&1 || { echo "bench g$gph failed"; tail -3 $OUT/bench_g${gph}_$rnd.log; exit 1; }
    echo "graph=$gph $(grep -o '"value": [0-9.]*' $OUT/bench_g${gph}_$rnd.log | head -1)"
  done
done
