#!/bin/bash
# rocprofv3 kernel trace of the default bench (timeline + per-kernel stats) into $1.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=${1:-gpurun_out/prof_step}
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o bench -- \
  python bench.py --no-cpu-baseline > "$OUT/bench.log" 2>&1 || exit 1
grep '^{' "$OUT/bench.log" | cut -c1-200
