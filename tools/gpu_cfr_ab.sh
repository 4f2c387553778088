#!/bin/bash
# Fused cost-volume backward with its 7 offset rows unrolled (ab_cfr7, -DCFR_UNROLL=7) against
# the rolled loop (default): corr tests on the variant, flow_bench, step A/B.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=${1:-gpurun_out/cfr_ab}
mkdir -p $O
A=optical_flow_amd/_build/ab_cfr7/liboflow.so
OFLOW_LIB=$A timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_kernels.py -k "corr or cost_volume or concat" > $O/tests.log 2>&1; rc=$?; echo "tests rc $rc"; tail -2 $O/tests.log
case $rc in 0) ;; *) exit 1;; esac
for r in 1 2; do
timeout -k 10 200 python tools/flow_bench.py --flow-scale 0.3 > $O/flow_base_$r.txt 2>&1 || exit 1
OFLOW_LIB=$A timeout -k 10 200 python tools/flow_bench.py --flow-scale 0.3 > $O/flow_cfr7_$r.txt 2>&1 || exit 1
done
for f in $O/flow_*.txt; do echo "$f $(grep -o "'corr_bwd': [0-9.]*" $f) $(grep -o "level 3.*" $f | grep -o "corr_bwd \+[0-9.]* us")"; done
bash tools/gpu_ab.sh $O/ab 2 'b|OFLOW_ABX=0|--precision bf16 --batch 32' "b7|OFLOW_LIB=$A|--precision bf16 --batch 32" 'f|OFLOW_ABX=0|' "f7|OFLOW_LIB=$A|"
