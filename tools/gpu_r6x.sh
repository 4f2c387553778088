#!/bin/bash
# SQ / LDS counter passes over the 64-column split forms (enc.l2, enc.l3) against the
# 128-column form (dec3.c1): where do their wave-cycles go?
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
OUT=${1:-gpurun_out/r6x}
mkdir -p "$OUT"
timeout -k 10 120 python tools/conv_bench.py --reps 5 --only enc.l2,enc.l3,dec3.c1 > $OUT/conv_bench.txt 2>&1; cat $OUT/conv_bench.txt | grep -v amdgpu
bash tools/gpu_pmc_cmd.sh $OUT/pmc python tools/conv_bench.py --reps 3 --only enc.l2,enc.l3,dec3.c1 || exit 1
for i in 1 2 3 4; do python tools/pmc_sq.py $OUT/pmc/p$i/run_counter_collection.csv "conv_tile_x3" > $OUT/sq_p$i.txt 2>&1; done
cat $OUT/sq_p*.txt | head -120
