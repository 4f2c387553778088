#!/bin/bash
# conv_halo_b16 persistent form (of_set_tuning key 24): image-kernel tests with it on, the
# per-layer bench and the bf16 B=32 A/B.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=${1:-gpurun_out/persist}
mkdir -p "$OUT"
run() {
  local t=$1; shift
  timeout -k 10 "$t" "$@"; local rc=$?
  case $rc in 124|134|137|139) echo "step '$*' rc $rc: stopping"; exit $rc;; esac
  return $rc
}
OFLOW_TUNE=24=1 run 600 python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_kernels.py -k "b16i" > "$OUT/kern_p.log" 2>&1; echo "kernel tests (persist) rc $?"; tail -1 "$OUT/kern_p.log"
OFLOW_TUNE=24=1 run 600 python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_bf16_modules.py tests/test_gpu_fullsize.py::test_config3_384x512_b32_bf16 > "$OUT/mod_p.log" 2>&1; echo "module tests (persist) rc $?"; tail -1 "$OUT/mod_p.log"
OFLOW_TUNE=24=1 run 300 python tools/b16i_bench.py --batch 32 > "$OUT/b16i_p.txt" 2>&1; echo "b16i persist rc $?"; grep -v amdgpu "$OUT/b16i_p.txt" | head -6
B='--precision bf16 --batch 32 --steps 10 --warmup 3'
bash tools/gpu_ab.sh "$OUT/ab" 2 "tile||$B" "persist|OFLOW_TUNE=24=1|$B"
