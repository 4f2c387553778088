#!/bin/bash
# The wgrad side stream with CUs withheld from it (OFLOW_SIDE_CU_WITHHOLD,
# of_stream_create_cu_masked): whole-step A/B, bf16 B=32 and fp32 B=8.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/misc9
mkdir -p $O
OFLOW_SIDE_CU_WITHHOLD=32 timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_model.py -k "side or graph or train" > $O/tests.log 2>&1; rc=$?; echo "tests rc $rc"; tail -2 $O/tests.log
case $rc in 0|5) ;; *) exit 1;; esac
bash tools/gpu_ab.sh $O/ab 2 'b0|OFLOW_SIDE_CU_WITHHOLD=0|--precision bf16 --batch 32' \
  'b16|OFLOW_SIDE_CU_WITHHOLD=16|--precision bf16 --batch 32' \
  'b32|OFLOW_SIDE_CU_WITHHOLD=32|--precision bf16 --batch 32' \
  'b64|OFLOW_SIDE_CU_WITHHOLD=64|--precision bf16 --batch 32' \
  'f0|OFLOW_SIDE_CU_WITHHOLD=0|' 'f32|OFLOW_SIDE_CU_WITHHOLD=32|'
