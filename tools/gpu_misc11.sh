#!/bin/bash
# corr_fwd_blk's bf16 concat epilogue in 16-byte chunks (default) against the per-element form
# (ab_cat0, -DCAT16_CHUNK=0), and the batched GEMM / tile epilogues against the per-row ones
# (ab_epc0, -DEPC_BATCH=0): tests and step A/B.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/misc11
mkdir -p $O
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_kernels.py tests/test_gpu_bf16_modules.py -k "corr or concat or flow_module or gemm or bf16 or x3 or stem" > $O/tests.log 2>&1; rc=$?; echo "tests rc $rc"; tail -2 $O/tests.log
case $rc in 0) ;; *) exit 1;; esac
bash tools/gpu_ab.sh $O/ab 2 'b|OFLOW_MAIN_PRIO=0|--precision bf16 --batch 32' 'bcat0|OFLOW_LIB=optical_flow_amd/_build/ab_cat0/liboflow.so|--precision bf16 --batch 32' \
  'bepc0|OFLOW_LIB=optical_flow_amd/_build/ab_epc0/liboflow.so|--precision bf16 --batch 32' 'f|OFLOW_MAIN_PRIO=0|' 'fepc0|OFLOW_LIB=optical_flow_amd/_build/ab_epc0/liboflow.so|'
