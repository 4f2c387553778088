#!/bin/bash
# conv_tile_ws: parity test, per-layer A/B against conv_tile_bf16 (key 12 = 0 / 2), bf16 bench A/B.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=${1:-gpurun_out/ws}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -v -k "conv_ws_forms" --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; grep -E "passed|failed|Error|rel_l2" "$OUT/pytest.log" | tail -20; [ $rc -ne 0 ] && exit $rc
for t in 0 2; do
  timeout -k 10 200 python tools/conv_bench.py --bf16 --reps 10 --tune 12=$t --only dec3,dec2,dec1,enc.l3,enc.l4 > "$OUT/cb_$t.txt" 2>&1 || { tail -5 "$OUT/cb_$t.txt"; exit 1; }
  echo "== tune 12=$t"; grep -v amdgpu.ids "$OUT/cb_$t.txt"
done
for t in 0 2; do
  timeout -k 10 300 python bench.py --precision bf16 --batch 32 --steps 10 --warmup 3 --no-cpu-baseline --tune 12=$t > "$OUT/bench_$t.log" 2>&1 || { tail -5 "$OUT/bench_$t.log"; exit 1; }
  grep '^{' "$OUT/bench_$t.log" | cut -c1-300
done
