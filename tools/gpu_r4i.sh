#!/bin/bash
# Round 4: bf16 B=32 A/B -- b16i on smaller grids (decoder level 1), cost-volume df1 on the
# side stream vs the fused backward on the main stream.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
A='--precision bf16 --batch 32 --steps 10 --warmup 3'
bash tools/gpu_ab.sh gpurun_out/r4i 2 "base||$A" "min128|OFLOW_B16I_MIN_TILES=128|$A" \
  "min64|OFLOW_B16I_MIN_TILES=64|$A" "fusedcorr|OFLOW_CORR_DF1_SIDE=0|$A"
