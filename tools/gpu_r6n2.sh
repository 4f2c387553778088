#!/bin/bash
# the N = 2 path on one GPU (both ranks on device 0, tools/same_gpu.py): the C-ABI RCCL
# communicator first, then the gloo TorchComm; and the BN training-mode step at N = 2
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
OUT=${1:-gpurun_out/r6n2}
mkdir -p "$OUT"
export OFLOW_COMM_TIMEOUT=60
L="python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1"
timeout -k 10 240 $L --master-port 29531 tools/same_gpu.py bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/bench_rccl.log 2>&1; r=$?
echo "rccl rc $r"; grep -E '^\{|Error|error|warn' $OUT/bench_rccl.log | cut -c1-300 | head -8
[ $r -eq 124 ] || [ $r -eq 137 ] && exit $r
OFLOW_DP_COMM=torch timeout -k 10 240 $L --master-port 29532 tools/same_gpu.py bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/bench_torch.log 2>&1; r=$?
echo "torch rc $r"; grep -E '^\{|Error|error|warn' $OUT/bench_torch.log | cut -c1-300 | head -8
exit 0
