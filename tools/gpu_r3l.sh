#!/bin/bash
# full GPU suite + 2 fp32 benches
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=${1:-gpurun_out/r3l}
mkdir -p "$OUT"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_all.log" 2>&1
rc=$?
grep -E "FAILED|ERROR|Error" "$OUT/pytest_all.log" | head -8; tail -2 "$OUT/pytest_all.log"
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > "$OUT/bench_$i.log" 2>&1 || { echo bench failed; tail -5 "$OUT/bench_$i.log"; exit 1; }
grep '^{' "$OUT/bench_$i.log" | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('fp32', d['value'], d['ms_per_step'], r['frac'])"
done
