#!/bin/bash
# bf16 B=32 step A/B over the host-side switches (two rounds each).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=${1:-gpurun_out/r3q}
mkdir -p "$OUT"
b() { local tag=$1; shift; env "$@" timeout -k 10 300 python bench.py --no-cpu-baseline --precision bf16 --batch 32 --steps 15 --warmup 3 > "$OUT/b_$tag.log" 2>&1 || { echo bench $tag failed; tail -5 "$OUT/b_$tag.log"; return 1; }; echo "$tag $(grep -o '"value": [0-9.]*' $OUT/b_$tag.log)"; }
for r in 1 2; do
b def$r OFLOW_X=0 || exit 1
b df1side$r OFLOW_CORR_DF1_SIDE=1 || exit 1
b side1m$r OFLOW_SIDE_MAX_PIX=1048576 || exit 1
b bnside0$r OFLOW_BN_SIDE=0 || exit 1
done
