#!/bin/bash
# bf16 A/B: tall input-gradient tiles (key 18), per-mode one-plane GEMMs (key 16 = 6 default
# vs 7), after the kernel tests of the forms.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=${1:-gpurun_out/r3o}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "tall or gemm_b16 or stem_b16 or conv_bf16" --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; grep -E "FAILED|Error|passed|failed" "$OUT/pytest.log" | tail -5; [ $rc -ne 0 ] && exit $rc
b() { local tag=$1; shift; timeout -k 10 300 python bench.py --no-cpu-baseline --precision bf16 --batch 32 --steps 15 --warmup 3 "$@" > "$OUT/bench_$tag.log" 2>&1 || { echo bench $tag failed; tail -5 "$OUT/bench_$tag.log"; return 1; }; echo "$tag $(grep -o '"value": [0-9.]*' $OUT/bench_$tag.log)"; }
b def || exit 1
b t18 --tune 18=1 || exit 1
b k16_7 --tune 16=7 || exit 1
b def2 || exit 1
b t18b --tune 18=1 || exit 1
