#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/misc4
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_kernels.py -k b16i > gpurun_out/misc4/b16i_tests.log 2>&1; rc=$?; echo "b16i tests rc $rc"; tail -2 gpurun_out/misc4/b16i_tests.log
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 300 python tools/conv_bench.py > gpurun_out/misc4/conv_base.txt 2>&1 || exit 1
OFLOW_LIB=optical_flow_amd/_build/ab_x3abl16/liboflow.so timeout -k 10 300 python tools/conv_bench.py > gpurun_out/misc4/conv_abl16.txt 2>&1 || exit 1
echo conv ok
bash tools/gpu_pmc_flow4.sh gpurun_out/misc4/pmc
