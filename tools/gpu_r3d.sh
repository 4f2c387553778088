#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=${1:-gpurun_out/r3d}
mkdir -p "$OUT"
timeout -k 10 60 ./tools/probes/graph_event_probe > "$OUT/probe.log" 2>&1; echo "probe rc $?"; cat "$OUT/probe.log"
timeout -k 10 300 python -u -m pytest tests/test_gpu_graph.py -v -s --timeout 200 --timeout-method thread > "$OUT/pytest_graph.log" 2>&1
rc=$?
grep -E "passed|failed|FAILED|Error|replay|graph step" "$OUT/pytest_graph.log" | tail -30
exit $rc
