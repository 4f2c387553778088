#!/bin/bash
# GPU side of an A/B run: conv_bench on the default library and on every variant built by
# tools/ab_build.sh (optical_flow_amd/_build/ab_*/liboflow.so), restricted to --only layers.
#   tools/ab_conv.sh "dec3.c1,enc.l3" [reps]
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
ONLY=$1; REPS=${2:-10}
echo "== base"
timeout -k 10 120 python tools/conv_bench.py --reps $REPS --only "$ONLY" 2>&1 | grep -v amdgpu.ids || exit 1
for d in optical_flow_amd/_build/ab_*; do
  [ -f $d/liboflow.so ] || continue
  echo "== $(basename $d)"
  OFLOW_LIB=$d/liboflow.so timeout -k 10 120 python tools/conv_bench.py --reps $REPS --only "$ONLY" 2>&1 | grep -v amdgpu.ids || exit 1
done
