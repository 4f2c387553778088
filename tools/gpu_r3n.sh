#!/bin/bash
# narrow kernels (loads in flight, wgrad register prefetch), bf16 one-plane stem and implicit
# GEMMs: kernel tests, then fp32 B=8 and bf16 B=32 benches with A/B of keys 15 / 16.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=${1:-gpurun_out/r3n}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "conv_bf16 or stem or gemm_b16 or conv_fwd_bwd" --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; grep -E "FAILED|Error|passed|failed" "$OUT/pytest.log" | tail -5; [ $rc -ne 0 ] && exit $rc
b() { local tag=$1; shift; timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > "$OUT/bench_$tag.log" 2>&1 || { echo bench $tag failed; tail -5 "$OUT/bench_$tag.log"; return 1; }; echo "$tag $(grep -o '"value": [0-9.]*' $OUT/bench_$tag.log)"; }
b f32 --steps 20 --warmup 5 || exit 1
b bf16 --precision bf16 --batch 32 --steps 15 --warmup 3 || exit 1
b bf16_k16 --precision bf16 --batch 32 --steps 15 --warmup 3 --tune 16=0 || exit 1
b bf16_k1516 --precision bf16 --batch 32 --steps 15 --warmup 3 --tune 15=0,16=0 || exit 1
b bf16b --precision bf16 --batch 32 --steps 15 --warmup 3 || exit 1
b bf16_il --precision bf16 --batch 32 --steps 15 --warmup 3 --tune 17=1 || exit 1
