#!/bin/bash
# The bf16 bench lines (config 3, B = 32; config 5 per GPU) into one directory.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=${1:-gpurun_out/bf16_lines}
mkdir -p "$OUT"
timeout -k 10 600 python bench.py --precision bf16 --batch 32 --cpu-steps 1 > "$OUT/bench_bf16.log" 2>&1 || { echo bf16 failed; tail -5 "$OUT/bench_bf16.log"; exit 1; }
grep '^{' "$OUT/bench_bf16.log" | head -c 200; echo
timeout -k 10 600 python bench.py --precision bf16 --height 768 --width 1024 --batch 8 --no-cpu-baseline > "$OUT/bench_cfg5.log" 2>&1 || { echo cfg5 failed; exit 1; }
grep '^{' "$OUT/bench_cfg5.log" | head -c 200; echo
