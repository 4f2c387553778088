#!/bin/bash
# A/B of of_set_tuning switches in one process tree on one box: for each "tag:k=v,..." variant
# (and the default), conv_bench on $1 layers and the whole-step bench, $2 rounds interleaved.
#   tools/gpu_abtune.sh "dec3.c1,enc.l3" 2 "old:4=0" "novec:3=0"
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
ONLY=$1; R=$2; shift 2
for i in $(seq $R); do
  for v in "base:" "$@"; do
    tag=${v%%:*}; tune=${v#*:}
    echo "== $tag round $i"
    if [ -n "$ONLY" ]; then OFLOW_TUNE=$tune timeout -k 10 120 python tools/conv_bench.py --reps 10 --only "$ONLY" 2>&1 | grep -v amdgpu.ids || exit 1; fi
    OFLOW_TUNE=$tune timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --timing-steps 0 2>/dev/null | grep '^{' | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench', d['value'], d['ms_per_step'])" || exit 1
  done
done
