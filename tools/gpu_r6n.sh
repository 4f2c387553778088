#!/bin/bash
# graph race probe with the side streams switched off one by one (one-queue graph executor)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
OUT=${1:-gpurun_out/r6n}
mkdir -p "$OUT"
p() {  # tag, env..., then probe args after --
  local tag=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  echo "=== $tag: ${envs[*]} $*" >> "$OUT/probe.log"
  env DEBUG_HIP_FORCE_GRAPH_QUEUES=1 "${envs[@]}" timeout -k 10 200 python -u tools/graph_race_probe.py "$@" 2>&1 | grep -v "amdgpu.ids" >> "$OUT/probe.log"
  local r=${PIPESTATUS[0]}; echo "$tag rc $r"; return $r
}
p train_nobnside OFLOW_BN_SIDE=0 -- fp32 training || exit 1
p train_nowgside OFLOW_SIDE_MAX_PIX=0 -- fp32 training || exit 1
p train_noside OFLOW_SIDE_MAX_PIX=0 OFLOW_BN_SIDE=0 OFLOW_PROJ_SIDE=0 -- fp32 training || exit 1
p inf_nowgside OFLOW_SIDE_MAX_PIX=0 -- fp32 inference || exit 1
p inf_nobnside OFLOW_BN_SIDE=0 -- fp32 inference || exit 1
grep -E "^===|gradients differ|^   " "$OUT/probe.log" | head -120
