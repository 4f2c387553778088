#!/bin/bash
# single-stream capture vs eager: with / without the shared FlowGrad pool
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
OUT=${1:-gpurun_out/r6q}
mkdir -p "$OUT"
for v in 0 1; do
  echo "=== PROBE_CLEAR_POOL=$v" >> "$OUT/probe.log"
  PROBE_CLEAR_POOL=$v timeout -k 10 200 python -u tools/graph_race_probe.py fp32 inference 2>&1 | grep -v amdgpu.ids >> "$OUT/probe.log"; echo "clear=$v rc ${PIPESTATUS[0]}"
done
grep -E "===|differ|^   " "$OUT/probe.log" | head -40
