#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
for co in 96 128; do
echo "== default $co"; timeout -k 10 120 python tools/probes/dbg_ws.py $co 2>&1 | grep -v amdgpu.ids
echo "== perwave $co"; OFLOW_LIB=optical_flow_amd/_build/ab_perwave/liboflow.so timeout -k 10 120 python tools/probes/dbg_ws.py $co 2>&1 | grep -v amdgpu.ids | grep -E "bad frac|unwritten|by channel" -A3
done
