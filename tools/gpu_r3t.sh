#!/bin/bash
# bf16 fragment prefetch (keys 17 / 20) + cost-volume 8x16 tiles (key 19) + df1 default:
# kernel / model tests, then bf16 B=32 and fp32 B=8 A/B.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=${1:-gpurun_out/r3t}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -m gpu -x -q -k "prefetch or conv_bf16 or cost_volume or corr or flow_net or wgrad_tile" --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; grep -E "FAILED|Error|passed|failed" "$OUT/pytest.log" | tail -5; [ $rc -ne 0 ] && exit $rc
b() { local tag=$1; shift; env "$@" timeout -k 10 300 python bench.py --no-cpu-baseline $ARGS > "$OUT/b_$tag.log" 2>&1 || { echo bench $tag failed; tail -5 "$OUT/b_$tag.log"; return 1; }; echo "$tag $(grep -o '"value": [0-9.]*' $OUT/b_$tag.log)"; }
for r in 1 2; do
ARGS="--precision bf16 --batch 32 --steps 15 --warmup 3"
b bf16_$r OFLOW_X=0 || exit 1
ARGS="--precision bf16 --batch 32 --steps 15 --warmup 3 --tune 17=0,20=0"
b bf16_nopf_$r OFLOW_X=0 || exit 1
ARGS="--precision bf16 --batch 32 --steps 15 --warmup 3 --tune 19=1"
b bf16_ty8_$r OFLOW_X=0 || exit 1
ARGS="--steps 20 --warmup 5"
b f32_$r OFLOW_X=0 || exit 1
ARGS="--steps 20 --warmup 5 --tune 19=1"
b f32_ty8_$r OFLOW_X=0 || exit 1
done
