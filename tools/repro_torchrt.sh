#!/bin/bash
# Run tools/repro_graph_rccl against the HIP runtime and RCCL that a torch process uses (the
# wheel's bundled ROCm 7.0.2 libamdhip64 / librccl, which liboflow.so also binds to inside
# python: same sonames) instead of /opt/rocm 7.2's: an alias directory in /tmp with the
# sonames the binary asks for, searched before its RUNPATH.
# usage: bash tools/repro_torchrt.sh <mode> <log>
TL=$(python -c "import os, torch; print(os.path.join(os.path.dirname(torch.__file__), 'lib'))")
D=$(mktemp -d /tmp/trt.XXXX)
for f in "$TL"/*.so*; do ln -sf "$f" "$D/"; done
ln -sf "$TL/libamdhip64.so" "$D/libamdhip64.so.7"
ln -sf "$TL/librccl.so" "$D/librccl.so.1"
LD_LIBRARY_PATH=$D ldd ./tools/repro_graph_rccl | grep -E "amdhip|rccl|hsa-runtime"
LD_LIBRARY_PATH=$D timeout -k 10 120 ./tools/repro_graph_rccl "$1"
