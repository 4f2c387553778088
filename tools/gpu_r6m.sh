#!/bin/bash
# graph race probe: captured step vs eager step, deterministic warp backward, with HIP's graph
# executor on one queue (topological order) -- fp32 / bf16, inference / training BN.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
OUT=${1:-gpurun_out/r6m}
mkdir -p "$OUT"
for cfg in "fp32 inference" "fp32 training" "bf16 inference"; do
  DEBUG_HIP_FORCE_GRAPH_QUEUES=1 timeout -k 10 240 python -u tools/graph_race_probe.py $cfg >> "$OUT/probe.log" 2>&1
  r=$?; echo "$cfg rc $r"; [ $r -eq 0 ] || exit $r
done
echo "--- default graph queues"; timeout -k 10 240 python -u tools/graph_race_probe.py fp32 inference >> "$OUT/probe.log" 2>&1; echo "default rc $?"
cat "$OUT/probe.log" | grep -v "^/opt\|amdgpu.ids"
