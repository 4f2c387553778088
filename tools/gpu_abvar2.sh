#!/bin/bash
# A/B of the in-tree library against a variant (OFLOW_LIB=$1): per-layer conv_bench (fp32) and
# the default bench, alternating twice.  Usage: tools/gpu_abvar2.sh VARIANT_SO [OUT] [conv_bench args]
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
V=$1; OUT=${2:-gpurun_out/abvar2}; shift 2; CB="$@"
mkdir -p "$OUT"
timeout -k 10 200 python tools/conv_bench.py --reps 10 --only dec3,dec2,enc.l3,enc.l4 $CB > "$OUT/cb_new.txt" 2>&1 || { tail -3 "$OUT/cb_new.txt"; exit 1; }
OFLOW_LIB=$V timeout -k 10 200 python tools/conv_bench.py --reps 10 --only dec3,dec2,enc.l3,enc.l4 $CB > "$OUT/cb_var.txt" 2>&1 || { tail -3 "$OUT/cb_var.txt"; exit 1; }
echo "== new"; grep -v amdgpu.ids "$OUT/cb_new.txt"; echo "== variant"; grep -v amdgpu.ids "$OUT/cb_var.txt"
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/b_new$r.log" 2>&1 || exit 1
  OFLOW_LIB=$V timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/b_var$r.log" 2>&1 || exit 1
  echo "round $r new $(grep -o '"value": [0-9.]*' $OUT/b_new$r.log) var $(grep -o '"value": [0-9.]*' $OUT/b_var$r.log)"
done
