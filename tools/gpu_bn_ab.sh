#!/bin/bash
# BN backward reductions with every load of a round issued together (buffer loads, default)
# against the pointer form (ab_bnold: -DMPB_BATCH=0 -DBNP_BATCH=0): the whole -m gpu suite,
# per-kernel rocprof stats of both, step A/B.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=${1:-gpurun_out/bn_ab}
mkdir -p $O
bash tools/gpu_tests_all.sh $O/tests || exit 1
grep -q " failed" $O/tests/pytest_gpu.log && exit 1
A=optical_flow_amd/_build/ab_bnold/liboflow.so
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_new -o run -- python bench.py --precision bf16 --batch 32 --no-cpu-baseline --steps 5 --warmup 3 --timing-steps 0 > $O/prof_new.log 2>&1 || exit 1
OFLOW_LIB=$A timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_old -o run -- python bench.py --precision bf16 --batch 32 --no-cpu-baseline --steps 5 --warmup 3 --timing-steps 0 > $O/prof_old.log 2>&1 || exit 1
for v in new old; do f=$(find $O/prof_$v -name "*kernel_stats.csv" | head -1); echo "$v"; grep -E "bn_act_bwd_partial|maxpool_bn" "$f" | cut -d, -f1-4 | cut -c1-150; done
bash tools/gpu_ab.sh $O/ab 2 'b|OFLOW_ABX=0|--precision bf16 --batch 32' "bold|OFLOW_LIB=$A|--precision bf16 --batch 32" 'f|OFLOW_ABX=0|' "fold|OFLOW_LIB=$A|"
