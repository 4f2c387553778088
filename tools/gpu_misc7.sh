#!/bin/bash
# Timing ablations of the fused cost-volume backward (CORR_ABL) and the warp backward
# (WARP_ABL) on tools/flow_bench.py: where their time goes.  Results of the ablated builds are
# wrong by design; only their timings are read.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/misc7
mkdir -p $O
timeout -k 10 200 python tools/flow_bench.py --flow-scale 0.3 > $O/flow_base.txt 2>&1 || exit 1
for v in corrabl1 corrabl2 corrabl4 corrabl7 warpabl1 warpabl2; do
  OFLOW_LIB=optical_flow_amd/_build/ab_$v/liboflow.so timeout -k 10 200 python tools/flow_bench.py --flow-scale 0.3 > $O/flow_$v.txt 2>&1 || exit 1
  echo "$v ok"
done
