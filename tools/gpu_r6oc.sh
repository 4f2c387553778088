#!/bin/bash
# own_window occupancy probe (of_set_tuning key 38: extra dynamic LDS per workgroup)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
OUT=${1:-gpurun_out/r6oc}
mkdir -p "$OUT"
for k in 0 4096 20000 45000 0; do
  OFLOW_TUNE=38=$k timeout -k 10 200 python tools/flow_bench.py --flow-scale 0.3 > $OUT/flow_k$k.txt 2>&1 || { echo "flow k$k failed"; exit 1; }
  echo "k$k"; grep -o "level . [^|]*|\|warp_bwd_det[^|]*|" $OUT/flow_k$k.txt | paste - - | head -3
done
