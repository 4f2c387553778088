#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
OUT=${1:-gpurun_out/r6s}
mkdir -p "$OUT"
for cfg in "fp32 inference" "fp32 training" "bf16 inference" "fp32 inference 384 512 8"; do
  timeout -k 10 240 python -u tools/uninit_probe.py $cfg 2>&1 | grep -v amdgpu.ids >> "$OUT/uninit.log"; echo "$cfg rc ${PIPESTATUS[0]}"
done
cat "$OUT/uninit.log" | grep -v Warning | head -150
