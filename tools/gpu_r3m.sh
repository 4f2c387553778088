#!/bin/bash
# Re-entry check: full GPU suite, then fp32 B=8 and bf16 B=32 benches.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=${1:-gpurun_out/r3m}
mkdir -p "$OUT"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_all.log" 2>&1
rc=$?
grep -E "FAILED|ERROR|Error" "$OUT/pytest_all.log" | head -8; tail -2 "$OUT/pytest_all.log"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > "$OUT/bench_f32.log" 2>&1 || { echo bench failed; tail -5 "$OUT/bench_f32.log"; exit 1; }
grep '^{' "$OUT/bench_f32.log" | head -c 400; echo
timeout -k 10 300 python bench.py --no-cpu-baseline --precision bf16 --batch 32 --steps 15 --warmup 3 > "$OUT/bench_bf16.log" 2>&1 || { echo bench failed; tail -5 "$OUT/bench_bf16.log"; exit 1; }
grep '^{' "$OUT/bench_bf16.log" | head -c 400; echo
for t in 2 3; do
  timeout -k 10 300 python bench.py --precision bf16 --batch 32 --steps 15 --warmup 3 --no-cpu-baseline --tune 12=$t > "$OUT/b_ws$t.log" 2>&1 || { tail -3 "$OUT/b_ws$t.log"; exit 1; }
  echo "tune 12=$t $(grep -o '"value": [0-9.]*' $OUT/b_ws$t.log)"
done
