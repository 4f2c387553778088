#!/bin/bash
# Kernel trace (durations) of tools/flow_bench.py per cost-volume form into $1.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=${1:-gpurun_out/flow_trace}
mkdir -p "$OUT"
for f in ${FORMS:-3 0}; do
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/f$f" -o run -- \
    python tools/flow_bench.py --reps 5 --corr-form $f > "$OUT/f$f.log" 2>&1 || exit 1
  grep -v amdgpu.ids "$OUT/f$f.log"
done
