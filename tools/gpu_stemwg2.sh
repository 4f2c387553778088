#!/bin/bash
# stem weight gradient: conv_wgrad_stem_x3 vs the fp32 GEMM, isolated (conv_bench) and in the step
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=${1:-gpurun_out/stemwg2}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_gpu_kernels.py -k "stem_wgrad" > "$OUT/pytest.log" 2>&1 || { tail -20 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for t in 14=1 14=0 14=1; do
  timeout -k 10 120 python tools/conv_bench.py --reps 20 --only enc.conv1 --tune $t 2>&1 | grep -v amdgpu.ids | tail -2 || exit 1
done
for r in 1 2; do
  for t in 14=1 14=0; do
    timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --warmup 5 --tune $t > "$OUT/b.log" 2>&1 || { tail -5 "$OUT/b.log"; exit 1; }
    grep '^{' "$OUT/b.log" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$t', d['value'], d['ms_per_step'], d['roofline']['per_kernel'].get('wgrad_stem_x3'))"
  done
done
