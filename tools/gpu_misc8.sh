#!/bin/bash
# The split 4-wave form without its halo-offset spills (X3_HREC) and the stem max-pool
# backward without dynamically indexed arrays: kernel tests, per-layer bench and step A/B
# against the X3_HREC=0 build.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/misc8
mkdir -p $O
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_kernels.py -k "x3 or maxpool or stem" > $O/tests.log 2>&1; rc=$?; echo "tests rc $rc"; tail -2 $O/tests.log
case $rc in 0) ;; *) exit 1;; esac
timeout -k 10 300 python tools/conv_bench.py > $O/conv_new.txt 2>&1 || exit 1
OFLOW_LIB=optical_flow_amd/_build/ab_hrec0/liboflow.so timeout -k 10 300 python tools/conv_bench.py > $O/conv_hrec0.txt 2>&1 || exit 1
echo conv ok
bash tools/gpu_ab.sh $O/ab 3 'new|OFLOW_MAIN_PRIO=0|' 'hrec0|OFLOW_LIB=optical_flow_amd/_build/ab_hrec0/liboflow.so|'
