#!/bin/bash
# graph-mode tests, graph vs eager bench A/B, then the whole -m gpu suite
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=${1:-gpurun_out/r3c}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_graph.py -v -s --timeout 200 --timeout-method thread > "$OUT/pytest_graph.log" 2>&1
rc=$?
grep -E "passed|failed|FAILED|Error|graph step|eager|weights rel" "$OUT/pytest_graph.log" | tail -30
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for g in 1 0 1 0; do
  timeout -k 10 300 python bench.py --graph $g --no-cpu-baseline --steps 20 --warmup 5 > "$OUT/bench_g$g.log" 2>&1 || { echo bench failed; tail -5 "$OUT/bench_g$g.log"; exit 1; }
  grep '^{' "$OUT/bench_g$g.log" | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('graph=$g', d['value'], d['ms_per_step'], r['frac'], r['launches_per_step'], r['avg_launch_ms'], r['window'])"
done
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_all.log" 2>&1
rc2=$?
grep -E "FAILED|ERROR" "$OUT/pytest_all.log" | head -5; tail -2 "$OUT/pytest_all.log"
exit $rc2
