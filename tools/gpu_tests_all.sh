#!/bin/bash
# The whole -m gpu suite (no -x: every failure listed) and smoke.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=${1:-gpurun_out/tests_all}
mkdir -p "$OUT"
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1
rc=$?
echo "pytest rc $rc"; tail -3 "$OUT/pytest_gpu.log"; grep -E "^FAILED|^ERROR" "$OUT/pytest_gpu.log" | head -20
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1; echo "smoke rc $?"; tail -2 "$OUT/smoke.log"
