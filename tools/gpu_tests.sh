#!/bin/bash
# The whole -m gpu suite (one process, per-test timeout), log under gpurun_out/$1.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=${1:-gpurun_out/tests}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?
grep -E "FAILED|ERROR" "$OUT/pytest_gpu.log" | head -5; tail -2 "$OUT/pytest_gpu.log"
exit $rc
