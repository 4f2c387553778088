#!/bin/bash
# Epilogue loads batched unguarded (epilogue_rows4c): conv_tile_bf16's per-block rows (default
# build; ab_tb0 = the round-2 one-row-at-a-time form) and the split kernels' X3_EPB = 4
# (ab_epb4; default 1).  Kernel tests, per-layer benches, step A/B.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/misc10
mkdir -p $O
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_kernels.py -k "bf16 or x3 or vec" > $O/tests.log 2>&1; rc=$?; echo "tests rc $rc"; tail -2 $O/tests.log
case $rc in 0) ;; *) exit 1;; esac
OFLOW_LIB=optical_flow_amd/_build/ab_epb4/liboflow.so timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_kernels.py -k "x3 or vec" > $O/tests_epb4.log 2>&1; rc=$?; echo "tests epb4 rc $rc"; tail -2 $O/tests_epb4.log
case $rc in 0) ;; *) exit 1;; esac
timeout -k 10 300 python tools/conv_bench.py > $O/conv_f32.txt 2>&1 || exit 1
OFLOW_LIB=optical_flow_amd/_build/ab_epb4/liboflow.so timeout -k 10 300 python tools/conv_bench.py > $O/conv_f32_epb4.txt 2>&1 || exit 1
timeout -k 10 300 python tools/conv_bench.py --bf16 > $O/conv_bf16.txt 2>&1 || exit 1
OFLOW_LIB=optical_flow_amd/_build/ab_epc0/liboflow.so timeout -k 10 300 python tools/conv_bench.py --bf16 > $O/conv_bf16_epc0.txt 2>&1 || exit 1
echo conv ok
bash tools/gpu_ab.sh $O/ab 2 'f|OFLOW_MAIN_PRIO=0|' 'fepb4|OFLOW_LIB=optical_flow_amd/_build/ab_epb4/liboflow.so|' 'fepc0|OFLOW_LIB=optical_flow_amd/_build/ab_epc0/liboflow.so|' \
  'b|OFLOW_MAIN_PRIO=0|--precision bf16 --batch 32' 'bepc0|OFLOW_LIB=optical_flow_amd/_build/ab_epc0/liboflow.so|--precision bf16 --batch 32'
