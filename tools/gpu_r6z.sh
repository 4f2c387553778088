#!/bin/bash
# 64-column conv_tile_x3 forms (of_set_tuning key 36): parity test, then interleaved benches
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
OUT=${1:-gpurun_out/r6z}
KEYS=${KEYS:-"0 1 2 3"}
mkdir -p "$OUT"
PT="python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 300 $PT tests/test_gpu_kernels_misc.py -k "bn64" > $OUT/tests.log 2>&1; r=$?
echo "tests rc $r"; grep -E "^FAILED|^E  |passed|failed" $OUT/tests.log | head -12
[ $r -eq 0 ] || exit $r
for rnd in 1 2; do
  for k in $KEYS; do
    OFLOW_TUNE=36=$k timeout -k 10 300 python bench.py --no-cpu-baseline $BENCH_ARGS > $OUT/bench_k${k}_$rnd.log 2>&1; r=$?
    [ $r -eq 0 ] || { echo "bench k$k rc $r"; tail -3 $OUT/bench_k${k}_$rnd.log; exit $r; }
    python - $OUT/bench_k${k}_$rnd.log $k <<'PY'
import json, sys
j = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
pk = j["roofline"]["per_kernel"]
sel = {k: v["ms_per_step"] for k, v in pk.items() if "<64" in k}
print("k%s %.1f pairs/s" % (sys.argv[2], j["value"]), "epe", j["parity"]["epe"], sel)
PY
  done
done
