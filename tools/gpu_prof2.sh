#!/bin/bash
# bench lines (fp32 B=8, bf16 B=32) + rocprof kernel stats of both + per-layer timing dumps.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=${1:-gpurun_out/p}
mkdir -p "$OUT"
OFLOW_TIMING_DUMP=$OUT/layers_fp32.json timeout -k 10 300 python bench.py > "$OUT/fp32.log" 2>&1 &&
OFLOW_TIMING_DUMP=$OUT/layers_bf16.json timeout -k 10 300 python bench.py --precision bf16 --batch 32 --no-cpu-baseline > "$OUT/bf16.log" 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_fp32" -o b -- python bench.py --no-cpu-baseline --steps 10 > "$OUT/fp32_prof.log" 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_bf16" -o b -- python bench.py --precision bf16 --batch 32 --no-cpu-baseline --steps 10 > "$OUT/bf16_prof.log" 2>&1
rc=$?
grep -h -o '"value": [0-9.]*' "$OUT"/fp32.log "$OUT"/bf16.log
exit $rc
