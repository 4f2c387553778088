#!/bin/bash
# tiled forward-image packing: parity tests, the model tests, bench lines and kernel traces
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=${1:-gpurun_out/r6pk}
mkdir -p "$OUT"
R="$GRAFT_REPO_ROOT/$OUT"
PT="python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $PT tests/test_gpu_kernels_misc.py tests/test_gpu_model.py -k "pack or flow_net or encoder or golden" > $OUT/tests.log 2>&1; r=$?
echo "tests rc $r"; grep -E "^FAILED|^E  |passed|failed" $OUT/tests.log | head -12
[ $r -eq 0 ] || exit $r
for p in fp32 bf16; do
  A=""; [ $p = bf16 ] && A="--precision bf16 --batch 32"
  timeout -k 10 300 python bench.py --no-cpu-baseline $A > $OUT/bench_$p.log 2>&1 || { echo "bench $p failed"; exit 1; }
  grep -o '"value": [0-9.]*' $OUT/bench_$p.log | head -1
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/prof_$p" -o b -- \
     python "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline --steps 4 --warmup 1 $A > "$R/prof_$p.log" 2>&1) || { echo "rocprof $p failed"; exit 1; }
  grep pack_many $OUT/prof_$p/b_kernel_stats.csv | cut -d, -f1-5
done
