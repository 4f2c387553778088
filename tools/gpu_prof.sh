#!/bin/bash
# rocprofv3 kernel-trace summary of the default bench (no CPU baseline), for profiles/.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=${1:-gpurun_out/prof}
mkdir -p "$OUT"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- \
  python bench.py --steps 10 --warmup 3 --no-cpu-baseline > "$OUT/bench.log" 2>&1
st=$?
echo "rocprof exit $st"
tail -2 "$OUT/bench.log"
find "$OUT" -name "*stats*" | head
exit $st
