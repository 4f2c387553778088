#!/bin/bash
# conv_tile_ws step probe (fwd, dgrad) and bf16 per-layer conv bench (key 12 = 0 / 2).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=${1:-gpurun_out/ws4}
mkdir -p "$OUT"
OFLOW_LIB=optical_flow_amd/_build/ab_stamp/liboflow.so timeout -k 10 120 python tools/ws_probe.py > "$OUT/probe_fwd.txt" 2>&1 || exit 1
OFLOW_LIB=optical_flow_amd/_build/ab_stamp/liboflow.so timeout -k 10 120 python tools/ws_probe.py --mode dgrad > "$OUT/probe_dgrad.txt" 2>&1 || exit 1
grep -v amdgpu.ids "$OUT/probe_fwd.txt" | head -30
for t in 0 2; do
  timeout -k 10 200 python tools/conv_bench.py --bf16 --reps 10 --tune 12=$t --only dec3,dec2,enc.l2 > "$OUT/cb_$t.txt" 2>&1 || { tail -5 "$OUT/cb_$t.txt"; exit 1; }
done
