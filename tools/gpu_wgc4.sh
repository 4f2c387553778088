#!/bin/bash
# cfg-4 weight gradient (32 x 64 channel blocks): tests, per-layer A/B, whole-step A/B.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/wgc4
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "wgrad_x3" > gpurun_out/wgc4/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/wgc4/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in 1 0 1; do
  echo "key11=$v"; timeout -k 10 120 python tools/conv_bench.py --reps 20 --only dec3.c3,dec3.c4,enc.l2 --tune 11=$v 2>&1 | grep -v amdgpu.ids || exit 1
done
timeout -k 10 120 python tools/conv_bench.py --reps 20 --tune 11=1 --shapes "dec2.c3:8,96,128,96,64,3,1;dec1.c3:8,48,64,96,64,3,1;dec0.c3:8,24,32,96,64,3,1" 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 120 python tools/conv_bench.py --reps 20 --tune 11=0 --shapes "dec2.c3:8,96,128,96,64,3,1;dec1.c3:8,48,64,96,64,3,1;dec0.c3:8,24,32,96,64,3,1" 2>&1 | grep -v amdgpu.ids || exit 1
bash tools/gpu_abenv.sh 2 "c4off:OFLOW_TUNE=11=0"
