#!/bin/bash
# stem weight-gradient kernel: parity tests, then A/B bench (key 14 via OFLOW_TUNING)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=${1:-gpurun_out/r3k}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_gpu_kernels.py -k "stem or gemm_x3_accuracy" > "$OUT/pytest.log" 2>&1
rc=$?
grep -E "PASS|FAIL|Error|rel_l2" "$OUT/pytest.log" | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_fullsize.py -k config2 > "$OUT/pytest2.log" 2>&1
rc=$?
tail -2 "$OUT/pytest2.log"
[ $rc -eq 0 ] || exit $rc
run() {
  local tag=$1; shift
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --warmup 5 "$@" > "$OUT/b_$tag.log" 2>&1 || { echo "bench $tag failed"; tail -5 "$OUT/b_$tag.log"; exit 1; }
  grep '^{' "$OUT/b_$tag.log" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', d['value'], d['ms_per_step'], d['roofline']['frac'])"
}
for r in 1 2; do
  run new_$r
  run old_$r --tune 14=0
done
