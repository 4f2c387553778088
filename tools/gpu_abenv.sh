#!/bin/bash
# Whole-step A/B over environment settings, $1 rounds interleaved:
#   tools/gpu_abenv.sh 3 "side:OFLOW_SIDE_MAX_PIX=100000000" "x:A=1 B=2"   (BENCH_ARGS: extra bench.py flags)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
R=$1; shift
for i in $(seq $R); do
  for v in "base:" "$@"; do
    tag=${v%%:*}; envs=${v#*:}
    out=$(env $envs timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline ${BENCH_ARGS:-} 2>/dev/null | grep '^{' | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], d['ms_per_step'], r['kernel'][11:60], r['frac'])") || exit 1
    echo "$tag round $i: $out"
  done
done
