#!/bin/bash
# Build a variant of liboflow.so with extra compile definitions for A/B timing:
#   tools/ab_build.sh NAME -DFOO=1 ...   ->  optical_flow_amd/_build/ab_NAME/liboflow.so
# Only conv_f32.hip is recompiled (set AB_SRCS to override); the other objects come from the
# main in-tree build (python optical_flow_amd/build.py).
# Run it with OFLOW_LIB=optical_flow_amd/_build/ab_NAME/liboflow.so python tools/conv_bench.py
set -e
cd "$(dirname "$0")/.."
NAME=$1; shift
OUT=optical_flow_amd/_build/ab_$NAME
mkdir -p $OUT
SRCS=${AB_SRCS:-conv_f32.hip}
objs=()
pids=()
for s in optical_flow_amd/csrc/*.hip optical_flow_amd/csrc/*.cpp; do
  b=$(basename $s)
  if [[ " $SRCS " == *" $b "* ]]; then
    o=$OUT/$b.o
    rm -f $o
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 "$@" -x hip -c $s -o $o &
    pids+=($!)
  else
    o=optical_flow_amd/_build/$b.o
  fi
  objs+=($o)
done
for p in "${pids[@]}"; do wait "$p" || { echo "compile failed" >&2; exit 1; }; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/liboflow.so "${objs[@]}" -lz -lpthread -ldl
echo $OUT/liboflow.so
