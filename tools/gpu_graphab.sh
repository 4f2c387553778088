#!/bin/bash
# eager vs HIP-graph replay of the whole step (bench.py --graph), fp32 and bf16
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
OUT=${1:-gpurun_out/r6graph}
mkdir -p "$OUT"
for p in fp32 bf16; do
  A=""; [ $p = bf16 ] && A="--precision bf16 --batch 32"
  for rnd in 1 2; do
    for gph in 0 1; do
      timeout -k 10 300 python bench.py --no-cpu-baseline --graph $gph $A > $OUT/bench_${p}_g${gph}_$rnd.log 2>&1 || { echo "bench $p g$gph failed"; tail -3 $OUT/bench_${p}_g${gph}_$rnd.log; exit 1; }
      echo "$p graph=$gph $(grep -o '"value": [0-9.]*' $OUT/bench_${p}_g${gph}_$rnd.log | head -1) $(grep -o '"final_loss": [0-9.]*' $OUT/bench_${p}_g${gph}_$rnd.log | head -1)"
    done
  done
done
