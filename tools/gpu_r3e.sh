#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=${1:-gpurun_out/r3e}
mkdir -p "$OUT"
timeout -k 10 60 ./tools/probes/graph_event_probe > "$OUT/probe.log" 2>&1; echo "probe rc $?"; cat "$OUT/probe.log"
timeout -k 10 400 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_kernels.py -k "graph or b16 or bf16" -v -s --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?
grep -E "passed|failed|FAILED|Error|replay|rel_l2" "$OUT/pytest.log" | tail -40
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for k in 1 0; do
  timeout -k 10 300 python bench.py --precision bf16 --batch 32 --no-cpu-baseline --graph 0 --tune 12=$k,13=$k > "$OUT/bench_b16_$k.log" 2>&1 || { echo bench failed; tail -5 "$OUT/bench_b16_$k.log"; exit 1; }
  grep '^{' "$OUT/bench_b16_$k.log" | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('key12=$k', d['value'], d['ms_per_step'], r['kernel'], r['frac']); [print('  ', k, v) for k, v in r['per_kernel'].items() if 'tile' in k]"
done
exit $rc
