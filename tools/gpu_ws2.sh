#!/bin/bash
# conv_tile_ws iteration: parity test, stamp probe, per-layer A/B (key 12 = 0 / 2).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=${1:-gpurun_out/ws2}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -v -k "conv_ws_forms" --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; grep -E "passed|failed|Error" "$OUT/pytest.log" | tail -5; [ $rc -ne 0 ] && exit $rc
OFLOW_LIB=optical_flow_amd/_build/ab_stamp/liboflow.so timeout -k 10 120 python tools/ws_probe.py > "$OUT/probe_fwd.txt" 2>&1 || exit 1
OFLOW_LIB=optical_flow_amd/_build/ab_stamp/liboflow.so timeout -k 10 120 python tools/ws_probe.py --mode dgrad > "$OUT/probe_dgrad.txt" 2>&1 || exit 1
grep -v amdgpu.ids "$OUT/probe_fwd.txt" | head -42
grep "block" "$OUT/probe_dgrad.txt"
for t in 0 2; do
  timeout -k 10 200 python tools/conv_bench.py --bf16 --reps 10 --tune 12=$t --only dec3,dec2,dec1,enc.l3,enc.l4 > "$OUT/cb_$t.txt" 2>&1 || { tail -5 "$OUT/cb_$t.txt"; exit 1; }
  echo "== tune 12=$t"; grep -v amdgpu.ids "$OUT/cb_$t.txt" | head -8
done
