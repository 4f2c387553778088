#!/bin/bash
# Build a variant of liboflow.so with extra compile definitions for A/B timing:
#   tools/ab_build.sh NAME -DFOO=1 ...   ->  optical_flow_amd/_build/ab_NAME/liboflow.so
# Run it with OFLOW_LIB=optical_flow_amd/_build/ab_NAME/liboflow.so python tools/conv_bench.py
set -e
cd "$(dirname "$0")/.."
NAME=$1; shift
OUT=optical_flow_amd/_build/ab_$NAME
mkdir -p $OUT
objs=()
for s in optical_flow_amd/csrc/*.hip optical_flow_amd/csrc/*.cpp; do
  o=$OUT/$(basename $s).o
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 "$@" -x hip -c $s -o $o &
  objs+=($o)
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/liboflow.so "${objs[@]}"
echo $OUT/liboflow.so
