#!/bin/bash
# stem max-pool + BN backward with 2 pooled pixels in flight (MPB_UNROLL=2) vs 1 (ab_mpb1):
# its tests, then bf16 B=32 / fp32 B=8 A/B alternating.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=${1:-gpurun_out/r3v}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -m gpu -x -q -k "maxpool or flow_net" --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; grep -E "FAILED|Error|passed|failed" "$OUT/pytest.log" | tail -5; [ $rc -ne 0 ] && exit $rc
b() { local tag=$1; shift; env "$@" timeout -k 10 300 python bench.py --no-cpu-baseline $ARGS > "$OUT/b_$tag.log" 2>&1 || { echo bench $tag failed; tail -5 "$OUT/b_$tag.log"; return 1; }; echo "$tag $(grep -o '"value": [0-9.]*' $OUT/b_$tag.log)"; }
for r in 1 2; do
ARGS="--precision bf16 --batch 32 --steps 15 --warmup 3"
b bf16_u2_$r OFLOW_X=0 || exit 1
b bf16_u1_$r OFLOW_LIB=optical_flow_amd/_build/ab_mpb1/liboflow.so || exit 1
ARGS="--steps 20 --warmup 5"
b f32_u2_$r OFLOW_X=0 || exit 1
b f32_u1_$r OFLOW_LIB=optical_flow_amd/_build/ab_mpb1/liboflow.so || exit 1
done
