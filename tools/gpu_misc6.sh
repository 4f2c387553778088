#!/bin/bash
# The split input gradient's direct epilogue (of_set_tuning key 23 bit 1): kernel tests,
# per-layer conv bench and whole-step A/B against the per-pass transposes (23=1).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/misc6
mkdir -p $O
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_kernels.py -k "x3 or dgrad_add or maxpool or corr or warp" > $O/tests.log 2>&1; rc=$?; echo "tests rc $rc"; tail -3 $O/tests.log
case $rc in 0) ;; *) exit 1;; esac
timeout -k 10 300 python tools/conv_bench.py > $O/conv_d3.txt 2>&1 || exit 1
OFLOW_TUNE=23=1 timeout -k 10 300 python tools/conv_bench.py > $O/conv_d1.txt 2>&1 || exit 1
echo conv ok
bash tools/gpu_ab.sh $O/ab 3 'd3|OFLOW_TUNE=23=3|' 'd1|OFLOW_TUNE=23=1|'
