mkdir -p gpurun_out/r6f
bash tools/repro_torchrt.sh two-big > gpurun_out/r6f/cpp_two_big.log 2>&1; r=$?; echo "cpp two-big rc $r"; tail -3 gpurun_out/r6f/cpp_two_big.log; [ $r -eq 0 ] || exit $r
timeout -k 10 150 python -u tools/repro_graph_rccl_torch.py torch_big > gpurun_out/r6f/torch_big.log 2>&1; r=$?; echo "torch_big rc $r"; tail -3 gpurun_out/r6f/torch_big.log; [ $r -eq 0 ] || exit $r
timeout -k 10 150 python -u tools/repro_graph_rccl_torch.py oflow_big > gpurun_out/r6f/oflow_big.log 2>&1; r=$?; echo "oflow_big rc $r"; tail -3 gpurun_out/r6f/oflow_big.log; exit $r
