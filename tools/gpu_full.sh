#!/bin/bash
# Round-end style check: smoke, GPU tests, default bench, rocprof summary of the default bench.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=${1:-gpurun_out/full}
mkdir -p "$OUT"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
st=$?; echo "smoke exit $st"; tail -2 "$OUT/smoke.log"; [ $st -ne 0 ] && exit $st
timeout -k 10 900 python -m pytest tests -m gpu -q -rf -x > "$OUT/pytest_gpu.log" 2>&1
st=$?; echo "pytest exit $st"; tail -4 "$OUT/pytest_gpu.log"; [ $st -ne 0 ] && exit $st
timeout -k 10 600 python bench.py > "$OUT/bench.log" 2>&1
st=$?; grep '^{' "$OUT/bench.log"; [ $st -ne 0 ] && exit $st
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o bench -- \
  python bench.py > "$OUT/bench_prof.log" 2>&1
st=$?; echo "rocprof exit $st"; grep '^{' "$OUT/bench_prof.log" | head -c 300; echo
exit $st
