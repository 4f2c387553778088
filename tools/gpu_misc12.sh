#!/bin/bash
# The stem max-pool + BN backward on 2048 workgroups (default) against 512 (ab_mpb512).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/misc12
mkdir -p $O
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_kernels.py tests/test_gpu_model.py -k "maxpool or stem or encoder" > $O/tests.log 2>&1; rc=$?; echo "tests rc $rc"; tail -2 $O/tests.log
case $rc in 0) ;; *) exit 1;; esac
bash tools/gpu_ab.sh $O/ab 2 'b|OFLOW_MAIN_PRIO=0|--precision bf16 --batch 32' 'b512|OFLOW_LIB=optical_flow_amd/_build/ab_mpb512/liboflow.so|--precision bf16 --batch 32' \
  'f|OFLOW_MAIN_PRIO=0|' 'f512|OFLOW_LIB=optical_flow_amd/_build/ab_mpb512/liboflow.so|'
