#!/bin/bash
# Build an A/B variant of liboflow.so whose SRC (a csrc file name) comes from git revision REV:
#   tools/ab_prev.sh REV flow_ops.hip[,misc.hip...] [NAME]  ->  optical_flow_amd/_build/ab_NAME/liboflow.so
set -e
cd "$(dirname "$0")/.."
REV=$1; SRC=$2; NAME=${3:-prev}
OUT=optical_flow_amd/_build/ab_$NAME
mkdir -p $OUT
TMP=$(mktemp -d)
for f in ${SRC//,/ }; do git show $REV:optical_flow_amd/csrc/$f > $TMP/$f; done
objs=()
for s in optical_flow_amd/csrc/*.hip optical_flow_amd/csrc/*.cpp; do
  b=$(basename $s)
  if [[ ",$SRC," == *",$b,"* ]]; then
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I optical_flow_amd/csrc -x hip -c $TMP/$b -o $OUT/$b.o
    objs+=($OUT/$b.o)
  else
    objs+=(optical_flow_amd/_build/$b.o)
  fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/liboflow.so "${objs[@]}" -lz -lpthread
rm -rf $TMP
echo $OUT/liboflow.so
