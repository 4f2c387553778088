#!/bin/bash
# A/B: eager vs graph, with / without the weight-gradient side stream; graph tests
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=${1:-gpurun_out/r3g}
mkdir -p "$OUT"
for cfg in "0 1" "1 1" "1 0" "0 0" "0 1" "1 0"; do
  set -- $cfg
  timeout -k 10 300 python bench.py --graph $1 --side-stream $2 --no-cpu-baseline --steps 20 --warmup 5 > "$OUT/bench_g$1s$2.log" 2>&1 || { echo bench failed; tail -5 "$OUT/bench_g$1s$2.log"; exit 1; }
  grep '^{' "$OUT/bench_g$1s$2.log" | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('graph=$1 side=$2', d['value'], d['ms_per_step'], r['frac'], r['avg_launch_ms'])"
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_graph.py -q -s --timeout 200 --timeout-method thread > "$OUT/pytest_graph.log" 2>&1; echo "graph tests rc $?"; grep -E "passed|failed|replay" "$OUT/pytest_graph.log" | tail -16
