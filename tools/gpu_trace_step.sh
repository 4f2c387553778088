#!/bin/bash
# Kernel trace of a short bench run (fp32 default and bf16 B=32) for tools/timeline.py.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=${1:-gpurun_out/trace}
mkdir -p "$OUT"
R="$GRAFT_REPO_ROOT/$OUT"
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/f32" -o run -- \
  python "$GRAFT_REPO_ROOT/bench.py" --steps 6 --warmup 3 --no-cpu-baseline > "$R/f32.log" 2>&1) || exit 1
python tools/timeline.py $(ls $OUT/f32/*kernel_trace.csv | head -1) --steps 3 > $OUT/f32_timeline.txt || exit 1
head -60 $OUT/f32_timeline.txt
if [ "$2" = "bf16" ]; then
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/bf16" -o run -- \
  python "$GRAFT_REPO_ROOT/bench.py" --steps 6 --warmup 3 --precision bf16 --batch 32 --no-cpu-baseline > "$R/bf16.log" 2>&1) || exit 1
python tools/timeline.py $(ls $OUT/bf16/*kernel_trace.csv | head -1) --steps 3 > $OUT/bf16_timeline.txt || exit 1
fi
