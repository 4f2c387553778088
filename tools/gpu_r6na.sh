#!/bin/bash
# act'-source read ablation of the split 3x3 input gradients (of_set_tuning key 39; wrong
# results, timing only): the bound on what sign masks could save
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
OUT=${1:-gpurun_out/r6na}
mkdir -p "$OUT"
for rnd in 1 2; do
  for k in 0 1; do
    OFLOW_TUNE=39=$k timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench_k${k}_$rnd.log 2>&1 || { echo "bench k$k failed"; exit 1; }
    python - $OUT/bench_k${k}_$rnd.log $k <<'PY'
import json, sys
j = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
pk, pa = j["roofline"]["per_kernel"], j["roofline"]["per_kernel_alone"]
d = sum(v["ms_per_step"] for k, v in pk.items() if k.startswith("dgrad_tile_x3"))
da = sum(v["ms_per_step"] for k, v in pa.items() if k.startswith("dgrad_tile_x3"))
print("k%s %.1f pairs/s  dgrad_tile_x3 in step %.3f ms alone %.3f ms" % (sys.argv[2], j["value"], d, da))
PY
  done
done
