#!/bin/bash
# whole-step A/B over one environment variable: VAR=OFLOW_X VALS="a b" [BENCH_ARGS=...] OUT
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
OUT=${1:-gpurun_out/envab}
mkdir -p "$OUT"
for rnd in 1 2; do
  for v in $VALS; do
    env "$VAR=$v" timeout -k 10 300 python bench.py --no-cpu-baseline $BENCH_ARGS > $OUT/bench_${v}_$rnd.log 2>&1 || { echo "bench $v failed"; tail -3 $OUT/bench_${v}_$rnd.log; exit 1; }
    echo "$VAR=$v $(grep -o '"value": [0-9.]*' $OUT/bench_${v}_$rnd.log | head -1)"
  done
done
