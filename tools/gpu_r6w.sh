#!/bin/bash
# per-layer conv timings (one fully timed step, side streams on and off) and the torch-level
# copies of a step
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
OUT=${1:-gpurun_out/r6w}
mkdir -p "$OUT"
OFLOW_TIMING_DUMP=$OUT/dump_side.json timeout -k 10 300 python bench.py --no-cpu-baseline --steps 4 --timing-steps 1 > $OUT/bench_side.log 2>&1; echo "side rc $?"
OFLOW_TIMING_DUMP=$OUT/dump_alone.json timeout -k 10 300 python bench.py --no-cpu-baseline --steps 4 --timing-steps 1 --side-stream 0 > $OUT/bench_alone.log 2>&1; echo "alone rc $?"
timeout -k 10 300 python tools/copy_probe.py fp32 8 2>&1 | grep -v amdgpu.ids > $OUT/copies.txt; echo "copies rc $?"
cat $OUT/copies.txt | head -40
