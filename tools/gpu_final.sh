#!/bin/bash
# the final tree: the whole -m gpu suite, smoke(), and one default bench line
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
OUT=${1:-gpurun_out/final}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1 || { echo tests failed; grep -E "^FAILED|^ERROR" "$OUT/pytest_gpu.log" | head -10; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo smoke failed; tail -5 "$OUT/smoke.log"; exit 1; }
echo smoke ok
timeout -k 10 600 python bench.py > "$OUT/bench.log" 2>&1 || { echo bench failed; tail -5 "$OUT/bench.log"; exit 1; }
grep '^{' "$OUT/bench.log" | head -c 400; echo
