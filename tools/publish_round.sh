#!/bin/bash
# Copy one tools/gpu_round5.sh output directory into profiles/ as round $2's evidence:
# bench lines, rocprof summaries (+ kernel stats), PMC traffic, micro-benchmarks.
# bash tools/publish_round.sh gpurun_out/round3 r2
set -e
IN=$1; R=$2
cd "$(dirname "$0")/.."
j() { grep '^{' "$1" | tail -1; }
[ -f "$IN/bench.log" ] || { echo "no bench.log in $IN (part A only?)"; exit 0; }
j "$IN/bench.log" > profiles/${R}_bench.json
j "$IN/bench_f32mfma.log" > profiles/${R}_bench_f32mfma.json
j "$IN/bench_bf16.log" > profiles/${R}_bf16_bench.json
j "$IN/bench_cfg5.log" > profiles/${R}_cfg5_bench.json
cp "$IN/prof/bench_kernel_stats.csv" profiles/${R}_bench_kernel_stats.csv
cp "$IN/prof_bf16/bench_kernel_stats.csv" profiles/${R}_bf16_bench_kernel_stats.csv
python tools/make_summary.py "$IN/bench.log" "$IN/prof/bench_kernel_stats.csv" \
  "python bench.py --no-cpu-baseline" > profiles/${R}_summary.md
python tools/make_summary.py "$IN/bench_bf16.log" "$IN/prof_bf16/bench_kernel_stats.csv" \
  "python bench.py --precision bf16 --batch 32 --no-cpu-baseline" > profiles/${R}_bf16_summary.md
if [ -f "$IN/pmc_traffic.json" ]; then
  cp "$IN/pmc_traffic.json" profiles/pmc_traffic.json
else
  python tools/pmc_traffic.py "$IN/fetch/bench_counter_collection.csv" "$IN/write/bench_counter_collection.csv" 384 512 8
fi
[ -f "$IN/bench_atomic.log" ] && j "$IN/bench_atomic.log" > profiles/${R}_bench_atomic_warp.json
[ -f "$IN/bench_repeat.log" ] && j "$IN/bench_repeat.log" > profiles/${R}_bench_repeat.json
[ -f "$IN/timed_state_check.txt" ] && cp "$IN/timed_state_check.txt" profiles/${R}_timed_state_check.txt
for f in mfma_f32 mfma_bf16 mfma_cfg5; do
  [ -f "$IN/$f.md" ] && cp "$IN/$f.md" profiles/${R}_$f.md
done
for f in conv_bench conv_bench_bf16 conv_bench_f32mfma flow_bench flow_bench_offset21 x3_accuracy b16i_bench; do
  [ -f "$IN/$f.txt" ] && grep -v amdgpu.ids "$IN/$f.txt" > profiles/${R}_$f.txt
done
true
