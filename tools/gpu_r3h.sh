#!/bin/bash
# per-layer conv tables (single stream, so per-launch times are not stretched by overlap)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=${1:-gpurun_out/r3h}
mkdir -p "$OUT"
OFLOW_TIMING_DUMP=$OUT/tdump_f32.json timeout -k 10 300 python bench.py --steps 6 --warmup 3 --no-cpu-baseline --side-stream 0 --timing-steps 2 > "$OUT/bench_f32.log" 2>&1 || { tail -3 "$OUT/bench_f32.log"; exit 1; }
OFLOW_TIMING_DUMP=$OUT/tdump_bf16.json timeout -k 10 300 python bench.py --precision bf16 --batch 32 --steps 6 --warmup 3 --no-cpu-baseline --side-stream 0 --timing-steps 2 > "$OUT/bench_bf16.log" 2>&1 || { tail -3 "$OUT/bench_bf16.log"; exit 1; }
python tools/layer_table.py $OUT/tdump_f32.json 2 255 > $OUT/table_f32.txt
python tools/layer_table.py $OUT/tdump_bf16.json 2 1500 > $OUT/table_bf16.txt
head -5 $OUT/table_f32.txt; head -5 $OUT/table_bf16.txt
