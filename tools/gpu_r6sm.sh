#!/bin/bash
# fp32 sign masks: parity tests, then interleaved benches OFLOW_SMASK=1 / 0
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
OUT=${1:-gpurun_out/r6sm}
mkdir -p "$OUT"
PT="python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 400 $PT tests/test_gpu_kernels_misc.py -k "sign_masks" > $OUT/tests.log 2>&1; r=$?
echo "tests rc $r"; grep -E "^FAILED|^E  |passed|failed" $OUT/tests.log | head -12
[ $r -eq 0 ] || exit $r
for rnd in 1 2 3; do
  for k in 1 0; do
    OFLOW_SMASK=$k timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench_k${k}_$rnd.log 2>&1 || { echo "bench k$k failed"; tail -3 $OUT/bench_k${k}_$rnd.log; exit 1; }
    python - $OUT/bench_k${k}_$rnd.log $k <<'PY'
import json, sys
j = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
pk, pa = j["roofline"]["per_kernel"], j["roofline"]["per_kernel_alone"]
d = sum(v["ms_per_step"] for k, v in pk.items() if k.startswith("dgrad_tile_x3"))
da = sum(v["ms_per_step"] for k, v in pa.items() if k.startswith("dgrad_tile_x3"))
f = sum(v["ms_per_step"] for k, v in pa.items() if k.startswith("fwd_tile_x3"))
print("smask=%s %.1f pairs/s loss %.8f dgrad_x3 in step %.3f alone %.3f fwd_x3 alone %.3f" % (sys.argv[2], j["value"], j["final_loss"], d, da, f))
PY
  done
done
