#!/bin/bash
# whole-step A/B of one of_set_tuning key: KEY=37 VALS="0 1" bash tools/gpu_r6fz.sh OUT
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
OUT=${1:-gpurun_out/r6fz}
KEY=${KEY:-37}
VALS=${VALS:-"0 1"}
mkdir -p "$OUT"
for rnd in 1 2 3; do
  for k in $VALS; do
    OFLOW_TUNE=$KEY=$k timeout -k 10 300 python bench.py --no-cpu-baseline $BENCH_ARGS > $OUT/bench_k${k}_$rnd.log 2>&1 || { echo "bench k$k failed"; tail -3 $OUT/bench_k${k}_$rnd.log; exit 1; }
    grep -o '"value": [0-9.]*' $OUT/bench_k${k}_$rnd.log | head -1 | sed "s/^/k$k /"
  done
done
