#!/bin/bash
# graph-mode bench (eager A/B), its rocprof kernel trace, graph trajectory test
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=${1:-gpurun_out/r3f}
mkdir -p "$OUT"
for g in 1 0 1 0; do
  timeout -k 10 300 python bench.py --graph $g --no-cpu-baseline --steps 20 --warmup 5 > "$OUT/bench_g$g.log" 2>&1 || { echo bench failed; tail -5 "$OUT/bench_g$g.log"; exit 1; }
  grep '^{' "$OUT/bench_g$g.log" | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('graph=$g', d['value'], d['ms_per_step'], r['frac'], r['launches_per_step'], r['avg_launch_ms'], r['window'])"
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_graph.py -q -s --timeout 200 --timeout-method thread > "$OUT/pytest_graph.log" 2>&1; echo "graph tests rc $?"; grep -E "passed|failed|graph step" "$OUT/pytest_graph.log" | tail -12
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$OUT/prof" -o bench -- python "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline --steps 20 --warmup 5 > "$GRAFT_REPO_ROOT/$OUT/bench_prof.log" 2>&1; echo "rocprof rc $?"
