#!/bin/bash
# graph replay stream priority (OFLOW_GRAPH_REPLAY_PRIO: -1 default high, 0 normal, none: the
# current stream) against eager, fp32
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
OUT=${1:-gpurun_out/r6graph2}
mkdir -p "$OUT"
for rnd in 1 2; do
  for pr in eager -1 0 none; do
    if [ $pr = eager ]; then G=0; E=""; else G=1; E="OFLOW_GRAPH_REPLAY_PRIO=$pr"; fi
    env $E timeout -k 10 300 python bench.py --no-cpu-baseline --graph $G > $OUT/bench_${pr}_$rnd.log 2>&1 || { echo "bench $pr failed"; tail -3 $OUT/bench_${pr}_$rnd.log; exit 1; }
    echo "prio=$pr $(grep -o '"value": [0-9.]*' $OUT/bench_${pr}_$rnd.log | head -1)"
  done
done
