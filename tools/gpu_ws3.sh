#!/bin/bash
# bf16 B=32 bench A/B: conv_tile_ws fwd only (key 12 = 3) / fwd+dgrad (2) / off (0), twice.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=${1:-gpurun_out/ws3}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "conv_ws_forms or conv_bf16 or conv_x3" --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -2 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do for t in 0 3 2; do
  timeout -k 10 300 python bench.py --precision bf16 --batch 32 --steps 15 --warmup 3 --no-cpu-baseline --tune 12=$t > "$OUT/b_${t}_${r}.log" 2>&1 || { tail -3 "$OUT/b_${t}_${r}.log"; exit 1; }
  echo "round $r tune 12=$t $(grep -o '"value": [0-9.]*' $OUT/b_${t}_${r}.log)"
done; done
timeout -k 10 200 python tools/host_time.py --steps 10 2>&1 | grep -v amdgpu.ids | tail -5
