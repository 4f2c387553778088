#!/bin/bash
# Warp backward with 512 destination slots (default, 6 workgroups per CU) against 1024
# (ab_cap1k, 5 per CU): tests, flow_bench at flow scales 0.3 and 2, step A/B.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=${1:-gpurun_out/warpcap_ab}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_kernels.py -k "warp" > $O/tests.log 2>&1; rc=$?; echo "tests rc $rc"; tail -2 $O/tests.log
case $rc in 0) ;; *) exit 1;; esac
A=optical_flow_amd/_build/ab_cap1k/liboflow.so
for r in 1 2; do for fs in 0.3 2.0; do
timeout -k 10 200 python tools/flow_bench.py --flow-scale $fs > $O/flow_new_${fs}_$r.txt 2>&1 || exit 1
OFLOW_LIB=$A timeout -k 10 200 python tools/flow_bench.py --flow-scale $fs > $O/flow_cap1k_${fs}_$r.txt 2>&1 || exit 1
done; done
for f in $O/flow_*.txt; do echo "$f $(grep -o "'warp_bwd': [0-9.]*" $f) $(grep -o "level 3.*" $f | grep -o "warp_bwd \+[0-9.]* us")"; done
bash tools/gpu_ab.sh $O/ab 2 'b|OFLOW_ABX=0|--precision bf16 --batch 32' "bold|OFLOW_LIB=$A|--precision bf16 --batch 32" 'f|OFLOW_ABX=0|' "fold|OFLOW_LIB=$A|"
