#!/bin/bash
# Round-4 checks on one box: b16i kernel tests (persistent fixture), the corr_bwd_fused fix
# (A/B lib: tests + flow_bench), flow-kernel PMC passes, the fp32 x3 epilogue ablation, and
# the bf16 df1-stream A/B.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/misc4
mkdir -p $O
FIX=optical_flow_amd/_build/ab_flowfix/liboflow.so
st() { case $1 in 124|134|137|139) echo "fatal rc $1"; exit $1;; esac; }
OFLOW_LIB=$FIX timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_kernels.py -k "corr or warp or maxpool" > $O/corrfix_tests.log 2>&1; rc=$?; echo "corrfix tests rc $rc"; tail -2 $O/corrfix_tests.log; st $rc
timeout -k 10 200 python tools/flow_bench.py > $O/flow_base.txt 2>&1 || exit 1
OFLOW_LIB=$FIX timeout -k 10 200 python tools/flow_bench.py > $O/flow_fix.txt 2>&1 || exit 1
echo flow ok
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_kernels.py -k b16i > $O/b16i_tests.log 2>&1; rc=$?; echo "b16i tests rc $rc"; tail -2 $O/b16i_tests.log; st $rc
bash tools/gpu_pmc_flow4.sh $O/pmc || exit 1
echo pmc ok
bash tools/gpu_ab.sh $O/ab 2 'side|OFLOW_CORR_DF1_SIDE=1|--precision bf16 --batch 32' \
  'fixside|OFLOW_LIB='$FIX'|--precision bf16 --batch 32' \
  'fixfused|OFLOW_CORR_DF1_SIDE=0 OFLOW_LIB='$FIX'|--precision bf16 --batch 32' \
  'fixprio|OFLOW_MAIN_PRIO=1 OFLOW_LIB='$FIX'|--precision bf16 --batch 32' \
  'fixmin128|OFLOW_B16I_MIN_TILES=128 OFLOW_LIB='$FIX'|--precision bf16 --batch 32' \
  'f32|OFLOW_MAIN_PRIO=0|' 'f32fix|OFLOW_LIB='$FIX'|' 'f32fixprio|OFLOW_MAIN_PRIO=1 OFLOW_LIB='$FIX'|'
