#!/bin/bash
# cost-volume backward on 8 x 16 tiles (key 19) and the per-precision df1 side stream:
# kernel / model tests, then fp32 B=8 and bf16 B=32 A/B (two rounds).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=${1:-gpurun_out/r3s2}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -m gpu -x -q -k "cost_volume or corr or flow_net" --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; grep -E "FAILED|Error|passed|failed" "$OUT/pytest.log" | tail -5; [ $rc -ne 0 ] && exit $rc
b() { local tag=$1; shift; env "$@" timeout -k 10 300 python bench.py --no-cpu-baseline $ARGS > "$OUT/b_$tag.log" 2>&1 || { echo bench $tag failed; tail -5 "$OUT/b_$tag.log"; return 1; }; echo "$tag $(grep -o '"value": [0-9.]*' $OUT/b_$tag.log)"; }
for r in 1 2; do
ARGS="--steps 20 --warmup 5"
b f32_$r OFLOW_X=0 || exit 1
ARGS="--steps 20 --warmup 5 --tune 19=1"
b f32_ty8_$r OFLOW_X=0 || exit 1
ARGS="--precision bf16 --batch 32 --steps 15 --warmup 3"
b bf16_$r OFLOW_X=0 || exit 1
b bf16_df1off_$r OFLOW_CORR_DF1_SIDE=0 || exit 1
ARGS="--precision bf16 --batch 32 --steps 15 --warmup 3 --tune 19=1"
b bf16_ty8_$r OFLOW_X=0 || exit 1
done
