#!/bin/bash
# kernel trace of the flow micro-benchmark: the deterministic warp backward's kernels one by one
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=${1:-gpurun_out/r6fy}
mkdir -p "$OUT"
R="$GRAFT_REPO_ROOT/$OUT"
(cd /tmp && OFLOW_TUNE=37=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/prof" -o fb -- \
  python "$GRAFT_REPO_ROOT/tools/flow_bench.py" --flow-scale 0.3 > "$R/fb.log" 2>&1) || { echo rocprof failed; exit 1; }
echo ok
