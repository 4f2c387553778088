#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "stem or conv_fwd_bwd or gemm_x3 or vec_epilogue" > gpurun_out/pytest_stem.log 2>&1 || { tail -40 gpurun_out/pytest_stem.log; exit 1; }
tail -2 gpurun_out/pytest_stem.log
for v in "OFLOW_STEM_X3=1" "OFLOW_TUNE=8=2" "OFLOW_STEM_X3=0"; do echo "$v"; env $v timeout -k 10 120 python tools/conv_bench.py --reps 10 --only enc.conv1 2>&1 | grep -v amdgpu.ids || exit 1; done
bash tools/gpu_abenv.sh 2 "fp32stem:OFLOW_STEM_X3=0" "stem64:OFLOW_TUNE=8=2"
