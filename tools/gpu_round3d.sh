#!/bin/bash
# Round-3 bf16 evidence re-taken after bench.py named the bf16 kernels' prefetch template
# argument (roofline symbol / PMC traffic lookup): bf16 B=32 bench (CPU baseline on 1 step),
# its rocprofv3 kernel-trace summary, and config 5.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=${1:-gpurun_out/round3d}
mkdir -p "$OUT"
R="$GRAFT_REPO_ROOT/$OUT"
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; }
run 600 python bench.py --precision bf16 --batch 32 --cpu-steps 1 > "$OUT/bench_bf16.log" 2>&1 || { echo bench bf16 failed; tail -5 "$OUT/bench_bf16.log"; exit 1; }
grep '^{' "$OUT/bench_bf16.log" | head -c 300; echo
(cd /tmp && run 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/prof_bf16" -o bench -- \
  python "$GRAFT_REPO_ROOT/bench.py" --precision bf16 --batch 32 --no-cpu-baseline > "$R/bench_bf16_prof.log" 2>&1) || { echo rocprof bf16 failed; exit 1; }
run 600 python bench.py --precision bf16 --height 768 --width 1024 --batch 8 --no-cpu-baseline > "$OUT/bench_cfg5.log" 2>&1 || { echo cfg5 bench failed; tail -5 "$OUT/bench_cfg5.log"; exit 1; }
grep '^{' "$OUT/bench_cfg5.log" | head -c 300; echo
echo done
