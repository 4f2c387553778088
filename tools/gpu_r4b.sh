#!/bin/bash
# Round 4: conv_halo_b16 per-layer A/B + the BN gamma guard test (verbose errors).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=${1:-gpurun_out/r4b}
mkdir -p "$OUT"
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; }
run 300 python tools/b16i_bench.py --batch 32 > "$OUT/b16i_b32.txt" 2>&1; echo "b16i b32 rc $?"; cat "$OUT/b16i_b32.txt" | grep -v amdgpu.ids
run 300 python tools/b16i_bench.py --batch 8 > "$OUT/b16i_b8.txt" 2>&1; echo "b16i b8 rc $?"; cat "$OUT/b16i_b8.txt" | grep -v amdgpu.ids
run 300 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread "tests/test_gpu_model.py::test_bn_gamma_near_zero" "tests/test_gpu_model.py::test_resnet_block_bn_guard" "tests/test_gpu_model.py::test_resnet_layer_simple" > "$OUT/bn.log" 2>&1; echo "bn rc $?"
grep -E "rel_l2|PASS|FAIL|Error" "$OUT/bn.log" | head -80
