#!/bin/bash
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=${1:-gpurun_out/cb}
mkdir -p "$OUT"
timeout -k 10 600 python tools/conv_bench.py --reps 10 > "$OUT/conv_bench.log" 2>&1
st=$?; cat "$OUT/conv_bench.log" | grep -v amdgpu.ids; [ $st -ne 0 ] && exit $st
OFLOW_TIMING_DUMP="$OUT/timing.json" timeout -k 10 600 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > "$OUT/bench.log" 2>&1
st=$?; grep '^{' "$OUT/bench.log" | head -c 600; exit $st
