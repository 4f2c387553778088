"""Run a script as one of several ranks that all use GPU 0 (LOCAL_RANK forced to 0 before
anything touches the GPU): the N > 1 code path -- rendezvous, the communicator vote and
self-test, the bucketed gradient all-reduce, BN statistics averaging, the max-over-ranks timing
-- exercised on a one-GPU box.  The ranks share one device, so the timing says nothing about
scaling.
  python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \
      --master-port 29533 tools/same_gpu.py bench.py --gpus 2 --steps 3 --warmup 1"""
import os
import runpy
import sys

os.environ["LOCAL_RANK"] = "0"
script = sys.argv[1]
sys.argv = sys.argv[1:]
sys.path.insert(0, os.path.dirname(os.path.abspath(script)))
runpy.run_path(script, run_name="__main__")
