"""Reproducer of the graph-replay segfault (late round 5): a captured step,
then a one-rank RCCL communicator that all-reduces on two streams (mode "stream"; "raw": the
second one made by hipStreamCreate; "close": destroyed after), then two more captured steps
-- the second one's replay segfaults in hipGraphLaunch.  python tools/repro_graph_rccl.py
stream_close"""
import os, sys
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
import torch
from optical_flow_amd import ops
from optical_flow_amd.comm import RcclComm
from test_gpu_graph import test_graph_steps_vs_oracle, _graph_vs_eager
mode = sys.argv[1]
test_graph_steps_vs_oracle()
comm = RcclComm(0, 1)
x = torch.randn(1 << 20, device="cuda")
comm.allreduce_(x)
if "stream" in mode:
    if "raw" in mode:
        import ctypes
        hip = ctypes.CDLL("libamdhip64.so")
        h = ctypes.c_void_p()
        assert hip.hipStreamCreate(ctypes.byref(h)) == 0
        s = torch.cuda.ExternalStream(h.value)
    else:
        s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        comm.allreduce_(x[: 12345])
    torch.cuda.current_stream().wait_stream(s)
torch.cuda.synchronize()
if "close" in mode:
    comm.close()
for det in (False, True):
    with ops.deterministic(det):
        _graph_vs_eager("fp32", None, det)
    print(mode, "det", det, "ok", flush=True)
