"""Which torch-level copies run in a train step (rocprof shows ~28 __amd_rocclr_copyBuffer
dispatches per fp32 step)?  Logs every aten copy / clone / contiguous-copy / cat / fill the
step dispatches, with shapes and the Python frame that issued it.
python tools/copy_probe.py [fp32|bf16] [B]"""
import collections
import os
import sys
import traceback

sys.path.insert(0, os.getcwd())
import torch  # noqa: E402
from torch.utils._python_dispatch import TorchDispatchMode  # noqa: E402

from optical_flow_amd.data import synthetic_batch  # noqa: E402
from optical_flow_amd.model import FlowNet  # noqa: E402
from optical_flow_amd.train import KerasAdam, Trainer  # noqa: E402

prec = sys.argv[1] if len(sys.argv) > 1 else "fp32"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 8
H, W = 384, 512
WATCH = ("copy_", "clone", "_to_copy", "cat", "fill_", "zero_", "zeros", "add", "mul", "div",
         "index", "stack", "contiguous", "copy")


class Log(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.seen = collections.Counter()

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        name = str(func.overloadpacket.__name__)
        if any(w in name for w in WATCH):
            shapes = tuple(tuple(a.shape) for a in args if isinstance(a, torch.Tensor))
            fr = [f for f in traceback.extract_stack()[:-1] if "optical_flow_amd" in f.filename
                  or "bench" in f.filename]
            where = ("%s:%d" % (os.path.basename(fr[-1].filename), fr[-1].lineno)) if fr else "?"
            self.seen[(name, shapes[:2], where)] += 1
        return func(*args, **(kwargs or {}))


net = FlowNet(H, W, precision=prec)
tr = Trainer(net, KerasAdam(net.store))
batch = torch.from_numpy(synthetic_batch(B, H, W, seed=3)).cuda()
for i in range(2):
    tr.train_step(batch, i)
torch.cuda.synchronize()
log = Log()
with log:
    tr.train_step(batch, 2)
torch.cuda.synchronize()
for (name, shapes, where), n in sorted(log.seen.items(), key=lambda t: -t[1]):
    print("%3d x %-14s %-40s %s" % (n, name, str(shapes)[:40], where))
