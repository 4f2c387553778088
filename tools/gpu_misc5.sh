#!/bin/bash
# Round-4 follow-up on one box: bf16 defaults A/B (cost-volume df1 stream vs fused on the main
# stream, b16i heads from 128 tiles), the fp32 x3 epilogue ablation, flow-kernel PMC on the
# current build.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/misc5
mkdir -p $O
timeout -k 10 300 python tools/conv_bench.py > $O/conv_base.txt 2>&1 || exit 1
OFLOW_LIB=optical_flow_amd/_build/ab_x3abl16/liboflow.so timeout -k 10 300 python tools/conv_bench.py > $O/conv_abl16.txt 2>&1 || exit 1
echo conv ok
bash tools/gpu_pmc_flow4.sh $O/pmc || exit 1
echo pmc ok
bash tools/gpu_ab.sh $O/ab 2 'base|OFLOW_CORR_DF1_SIDE=1 OFLOW_B16I_MIN_TILES=256|--precision bf16 --batch 32' \
  'fused128|OFLOW_CORR_DF1_SIDE=0 OFLOW_B16I_MIN_TILES=128|--precision bf16 --batch 32' \
  'side128|OFLOW_CORR_DF1_SIDE=1 OFLOW_B16I_MIN_TILES=128|--precision bf16 --batch 32' \
  'fused64|OFLOW_CORR_DF1_SIDE=0 OFLOW_B16I_MIN_TILES=64|--precision bf16 --batch 32'
