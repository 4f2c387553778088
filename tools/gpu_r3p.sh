#!/bin/bash
# Per-layer in-step conv timing dumps (fp32 B=8, bf16 B=32).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=${1:-gpurun_out/r3p}
mkdir -p "$OUT"
OFLOW_TIMING_DUMP=$OUT/td_f32.json timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/bench_f32.log 2>&1 || { tail -3 $OUT/bench_f32.log; exit 1; }
OFLOW_TIMING_DUMP=$OUT/td_bf16.json timeout -k 10 300 python bench.py --precision bf16 --batch 32 --steps 10 --warmup 3 --no-cpu-baseline > $OUT/bench_bf16.log 2>&1 || { tail -3 $OUT/bench_bf16.log; exit 1; }
echo done
