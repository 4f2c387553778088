#!/bin/bash
# Cost-volume forms: GPU tests of both forms, then the flow micro-bench per form.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=${1:-gpurun_out/corr}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "cost_volume or corr_concat" -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
for f in 3 0; do
  timeout -k 10 120 python tools/flow_bench.py --corr-form $f > "$OUT/flow_bench_$f.txt" 2>&1 || exit 1
  echo "form $f"; grep -v amdgpu.ids "$OUT/flow_bench_$f.txt"
done
