#!/bin/bash
# Round 4: rocprofv3 kernel-trace summaries of the bf16 B=32 and fp32 B=8 benches.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=${1:-gpurun_out/r4h}
mkdir -p "$OUT/bf16" "$OUT/fp32"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/bf16" -o run -- \
  python bench.py --precision bf16 --batch 32 --no-cpu-baseline > "$OUT/bf16/bench.log" 2>&1 || { echo "bf16 prof failed $?"; exit 1; }
echo "bf16 prof ok"; grep '^{' "$OUT/bf16/bench.log" | head -c 300; echo
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/fp32" -o run -- \
  python bench.py --no-cpu-baseline > "$OUT/fp32/bench.log" 2>&1 || { echo "fp32 prof failed $?"; exit 1; }
echo "fp32 prof ok"; grep '^{' "$OUT/fp32/bench.log" | head -c 300; echo
find "$OUT" -name "*stats*"
