#!/bin/bash
# tests -> conv microbench -> bench with per-layer timing dump -> rocprof kernel trace
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=${1:-gpurun_out/round}
mkdir -p "$OUT"
timeout -k 10 900 python -m pytest tests -m gpu -q -rf -x > "$OUT/pytest_gpu.log" 2>&1
st=$?; echo "pytest exit $st"; tail -6 "$OUT/pytest_gpu.log"; [ $st -ne 0 ] && exit $st
timeout -k 10 600 python tools/conv_bench.py --reps 10 > "$OUT/conv_bench.log" 2>&1
st=$?; grep -v amdgpu.ids "$OUT/conv_bench.log"; [ $st -ne 0 ] && exit $st
OFLOW_TIMING_DUMP="$OUT/timing.json" timeout -k 10 600 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > "$OUT/bench.log" 2>&1
st=$?; grep '^{' "$OUT/bench.log" | head -c 700; echo; [ $st -ne 0 ] && exit $st
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- \
  python bench.py --steps 10 --warmup 3 --no-cpu-baseline > "$OUT/bench_prof.log" 2>&1
st=$?; echo "rocprof exit $st"; exit $st
