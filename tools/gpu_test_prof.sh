#!/bin/bash
# GPU parity tests, then a rocprofv3 kernel-trace of the default bench.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=${1:-gpurun_out/prof}
mkdir -p "$OUT"
timeout -k 10 900 python -m pytest tests -m gpu -q -rf -x > "$OUT/pytest_gpu.log" 2>&1
st=$?
echo "pytest exit $st"; tail -15 "$OUT/pytest_gpu.log"
if [ $st -ne 0 ]; then exit $st; fi
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- \
  python bench.py --steps 10 --warmup 3 --no-cpu-baseline > "$OUT/bench.log" 2>&1
st=$?
echo "rocprof exit $st"; grep '^{' "$OUT/bench.log" | head -c 1500
exit $st
