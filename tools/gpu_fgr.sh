#!/bin/bash
# Flow-gradient routing: model / graph / bf16 module parity tests, then bench A/B (routing off).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=${1:-gpurun_out/fgr}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_graph.py tests/test_gpu_fullsize.py tests/test_gpu_bf16_modules.py tests/test_gpu_dist.py -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/b_new$r.log" 2>&1 || exit 1
  OFLOW_FLOW_GRAD_ROUTING=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/b_off$r.log" 2>&1 || exit 1
  echo "round $r new $(grep -o '"value": [0-9.]*' $OUT/b_new$r.log) off $(grep -o '"value": [0-9.]*' $OUT/b_off$r.log)"
done
