#!/bin/bash
# Round-end evidence in one GPU call: smoke, GPU tests, the default bench (fp32 config 2,
# with the CPU baseline), its rocprofv3 kernel-trace summary, FETCH_SIZE / WRITE_SIZE PMC
# passes, conv and flow micro-benchmarks, the bf16 (config 3) bench with its summary, and the
# fp32 bench / conv micro-bench with every conv on the fp32 MFMA kernels (OFLOW_F32_SPLIT=0).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=${1:-gpurun_out/round}
mkdir -p "$OUT"
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; }
run 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo smoke failed; tail -5 "$OUT/smoke.log"; exit 1; }
echo smoke ok
run 900 python -m pytest tests -m gpu -q -rf -x > "$OUT/pytest_gpu.log" 2>&1 || { echo pytest failed; tail -8 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
run 600 python bench.py > "$OUT/bench.log" 2>&1 || { echo bench failed; tail -5 "$OUT/bench.log"; exit 1; }
grep '^{' "$OUT/bench.log" | head -c 400; echo
run 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o bench -- \
  python bench.py --no-cpu-baseline > "$OUT/bench_prof.log" 2>&1 || { echo rocprof failed; exit 1; }
echo rocprof ok
run 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o bench -- \
  python bench.py --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/fetch.log" 2>&1 || { echo fetch failed; exit 1; }
run 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o bench -- \
  python bench.py --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/write.log" 2>&1 || { echo write failed; exit 1; }
echo pmc ok
run 300 python tools/conv_bench.py --reps 10 > "$OUT/conv_bench.txt" 2>&1 || exit 1
run 300 python tools/conv_bench.py --reps 10 --bf16 > "$OUT/conv_bench_bf16.txt" 2>&1 || exit 1
OFLOW_F32_SPLIT=0 run 300 python tools/conv_bench.py --reps 10 > "$OUT/conv_bench_f32mfma.txt" 2>&1 || exit 1
run 300 python tools/x3_accuracy.py > "$OUT/x3_accuracy.txt" 2>&1 || exit 1
run 300 python tools/flow_bench.py > "$OUT/flow_bench.txt" 2>&1 || exit 1
echo micro ok
run 600 python bench.py --precision bf16 --batch 32 --cpu-steps 0 > "$OUT/bench_bf16.log" 2>&1 || { echo bench bf16 failed; exit 1; }
grep '^{' "$OUT/bench_bf16.log" | head -c 300; echo
run 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_bf16" -o bench -- \
  python bench.py --precision bf16 --batch 32 --no-cpu-baseline > "$OUT/bench_bf16_prof.log" 2>&1 || { echo rocprof bf16 failed; exit 1; }
run 300 python tools/data_bench.py --batch 8 --out "$OUT/data_bench.json" > "$OUT/data_bench.log" 2>&1 || { echo data bench failed; exit 1; }
run 600 python bench.py --precision bf16 --height 768 --width 1024 --batch 8 --no-cpu-baseline > "$OUT/bench_cfg5.log" 2>&1 || { echo cfg5 bench failed; exit 1; }
grep '^{' "$OUT/bench_cfg5.log" | head -c 300; echo
OFLOW_F32_SPLIT=0 run 600 python bench.py --no-cpu-baseline > "$OUT/bench_f32mfma.log" 2>&1 || { echo f32mfma bench failed; exit 1; }
grep '^{' "$OUT/bench_f32mfma.log" | head -c 300; echo
echo done
