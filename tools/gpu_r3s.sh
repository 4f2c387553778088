#!/bin/bash
# Session check: the whole -m gpu suite, then the default bench and the bf16 B=32 bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=${1:-gpurun_out/r3s}
mkdir -p "$OUT"
bash tools/gpu_tests.sh "$OUT" || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/bench.log" 2>&1 || { tail -5 "$OUT/bench.log"; exit 1; }
grep '^{' "$OUT/bench.log" | cut -c1-400
timeout -k 10 300 python bench.py --precision bf16 --batch 32 --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/bench_bf16.log" 2>&1 || { tail -5 "$OUT/bench_bf16.log"; exit 1; }
grep '^{' "$OUT/bench_bf16.log" | cut -c1-400
