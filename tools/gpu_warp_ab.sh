#!/bin/bash
# Warp backward: corner rows for the flow gradient loaded after the scatter, two pixel groups
# at a time (default, 80 VGPRs) against: after the dout rows, all at once (ab_lpv1), one group
# at a time (ab_grp1), at the top (ab_wpv0). Tests, flow_bench, step A/B.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=${1:-gpurun_out/warp_ab2}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_kernels.py -k "warp" > $O/tests.log 2>&1; rc=$?; echo "tests rc $rc"; tail -2 $O/tests.log
case $rc in 0) ;; *) exit 1;; esac
B=optical_flow_amd/_build
for r in 1 2; do
timeout -k 10 200 python tools/flow_bench.py --flow-scale 0.3 > $O/flow_new_$r.txt 2>&1 || exit 1
for v in lpv1 grp1 wpv0; do
OFLOW_LIB=$B/ab_$v/liboflow.so timeout -k 10 200 python tools/flow_bench.py --flow-scale 0.3 > $O/flow_${v}_$r.txt 2>&1 || exit 1
done
done
for f in $O/flow_*.txt; do echo "$f $(grep -o "'warp_bwd': [0-9.]*" $f) $(grep -o "level 3.*" $f | grep -o "warp_bwd \+[0-9.]* us")"; done
bash tools/gpu_ab.sh $O/ab 2 'b|OFLOW_ABX=0|--precision bf16 --batch 32' "b1|OFLOW_LIB=$B/ab_lpv1/liboflow.so|--precision bf16 --batch 32" 'f|OFLOW_ABX=0|' "f1|OFLOW_LIB=$B/ab_lpv1/liboflow.so|"
