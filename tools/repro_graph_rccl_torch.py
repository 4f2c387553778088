"""Bisect the round-5 graph-replay host fault between torch and liboflow.
tools/repro_graph_rccl.cpp (HIP + RCCL, no torch) replays its graphs fine after a one-rank
communicator was used on two streams, on /opt/rocm 7.2 and on torch's bundled ROCm 7.0.2.
Here the same sequence runs inside torch with graphs of
  mode "torch": torch elementwise ops only (current stream + a forked side stream), or
  mode "oflow": liboflow launches only (of_fill / of_add_inplace, the side stream forked and
                joined with of_stream_wait, as the train step's capture does),
and the communicator is the C-ABI RcclComm used on the current stream and a second one, then
closed.  "<mode>_big": 64 such steps per graph (~320 nodes, the train step's order of
magnitude), each with a scratch tensor allocated inside the capture (torch's graph pool, as
the step's workspaces).  python tools/repro_graph_rccl_torch.py torch|oflow[_big]"""
import ctypes as C
import os
import sys

sys.path.insert(0, os.getcwd())
import torch  # noqa: E402

from optical_flow_amd import ops  # noqa: E402
from optical_flow_amd._lib import call  # noqa: E402
from optical_flow_amd.comm import RcclComm  # noqa: E402

mode = sys.argv[1]
REPS = 64 if mode.endswith("_big") else 1
mode = mode.replace("_big", "")
n = 1 << 22
a = torch.zeros(n, device="cuda")
b = torch.ones(n, device="cuda")
c = torch.ones(n, device="cuda")
side = torch.cuda.Stream()


def step():
    for _ in range(REPS):
        step1()
        if REPS > 1:
            t = torch.empty(1 << 16, device="cuda")
            call("of_fill", C.c_void_p(t.data_ptr()), 1.0, t.numel(),
                 C.c_void_p(torch.cuda.current_stream().cuda_stream))
            call("of_add_inplace", C.c_void_p(a.data_ptr()), C.c_void_p(t.data_ptr()),
                 t.numel(), C.c_void_p(torch.cuda.current_stream().cuda_stream))


def step1():
    cur = torch.cuda.current_stream()
    if mode == "torch":
        b.mul_(1.5).add_(1.0)
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            c.mul_(0.5).sub_(1.0)
        a.mul_(0.25).add_(b)
        cur.wait_stream(side)
        a.add_(c)
    else:
        P = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731
        call("of_add_inplace", P(b), P(a), n, C.c_void_p(cur.cuda_stream))
        ops.stream_wait(side, cur)
        call("of_fill", P(c), 0.5, n, C.c_void_p(side.cuda_stream))
        call("of_add_inplace", P(a), P(b), n, C.c_void_p(cur.cuda_stream))
        ops.stream_wait(cur, side)
        call("of_add_inplace", P(a), P(c), n, C.c_void_p(cur.cuda_stream))


def graph_and_replay(tag):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        step()                                   # warm-up off the default stream
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        step()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    print(mode, tag, "replayed", flush=True)


graph_and_replay("graph 0")
comm = RcclComm(0, 1)
x = torch.randn(1 << 20, device="cuda")
comm.allreduce_(x)
s2 = torch.cuda.Stream()
s2.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s2):
    comm.allreduce_(x[:12345])
torch.cuda.current_stream().wait_stream(s2)
torch.cuda.synchronize()
comm.close()
print(mode, "communicator used on two streams, closed", flush=True)
graph_and_replay("graph 1")
graph_and_replay("graph 2")
print(mode, "ok", flush=True)
