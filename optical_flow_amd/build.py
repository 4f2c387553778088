"""Build liboflow.so (gfx950) in-tree with hipcc.  No cmake/ninja: one hipcc -c per source in
parallel, one link.  The .so lives next to this file so gpurun snapshots carry it."""
from __future__ import annotations

import concurrent.futures as cf
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
BUILD = os.path.join(HERE, "_build")
LIB = os.path.join(HERE, "liboflow.so")
ARCH = os.environ.get("OFLOW_ARCH", "gfx950")
FLAGS = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=" + ARCH, "-Wall",
         "-Wno-unused-variable", "-Wno-unused-but-set-variable"]


def _hipcc():
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found: the HIP path cannot be built")


def sources():
    return sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC)
                  if f.endswith((".hip", ".cpp")))


def build(force: bool = False, verbose: bool = False) -> str:
    hipcc = _hipcc()
    os.makedirs(BUILD, exist_ok=True)
    srcs = sources()
    headers = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    headers.append(os.path.join(HERE, "..", "include", "oflow.h"))
    newest_hdr = max(os.path.getmtime(h) for h in headers)
    objs = []
    jobs = []
    for s in srcs:
        o = os.path.join(BUILD, os.path.basename(s) + ".o")
        objs.append(o)
        if force or not os.path.exists(o) or os.path.getmtime(o) < max(os.path.getmtime(s),
                                                                       newest_hdr):
            lang = ["-x", "hip"] if s.endswith(".hip") else ["-x", "hip"]
            jobs.append([hipcc] + FLAGS + lang + ["-c", s, "-o", o])

    def run(cmd):
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError("hipcc failed:\n" + " ".join(cmd) + "\n" + r.stdout + r.stderr)
        if verbose and (r.stdout or r.stderr):
            print(r.stdout + r.stderr, file=sys.stderr)

    workers = max(1, min(len(jobs), int(os.environ.get("MAX_JOBS", os.cpu_count() or 4)), 8))
    if jobs:
        with cf.ThreadPoolExecutor(workers) as ex:
            list(ex.map(run, jobs))
    if jobs or not os.path.exists(LIB) or os.path.getmtime(LIB) < max(os.path.getmtime(o)
                                                                        for o in objs):
        # link to a temporary name, then rename: a reader (or a snapshot of the tree) never
        # sees a half-written library
        tmp = LIB + ".tmp%d" % os.getpid()
        run([hipcc, "--offload-arch=" + ARCH, "-shared", "-fPIC", "-o", tmp] + objs + ["-lz", "-lpthread", "-ldl"])
        os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
