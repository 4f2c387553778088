#!/bin/bash
# Round 4: the whole -m gpu suite + smoke, then the fp32 A/B of the split forward's direct
# epilogue (key 23) and the bf16 A/B of the concat written as a bf16 image.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
bash tools/gpu_tests_all.sh gpurun_out/r4l || exit $?
F='--steps 20 --warmup 5'
bash tools/gpu_ab.sh gpurun_out/r4l/ab 2 "x3direct||$F" "x3pass|OFLOW_TUNE=23=0|$F"
B='--precision bf16 --batch 32 --steps 10 --warmup 3'
bash tools/gpu_ab.sh gpurun_out/r4l/ab16 2 "cat16||$B" "cat32|OFLOW_CONCAT_IMG16=0|$B"
