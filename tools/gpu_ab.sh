#!/bin/bash
# A/B of whole bench steps on ONE box, variants interleaved ROUNDS times (boxes differ by up to
# 10 %, so only same-call comparisons mean anything).  Replaces the round-2/3 one-off
# tools/gpu_r3*.sh scripts.
#
#   tools/gpu_ab.sh OUT ROUNDS 'label|ENV=V ENV2=V2|bench args' ['label|...|...' ...]
#
# e.g. tools/gpu_ab.sh gpurun_out/ab 3 'img|OFLOW_B16I=1|--precision bf16 --batch 32' \
#                                      'old|OFLOW_B16I=0|--precision bf16 --batch 32'
# Each variant: env assignments (space separated, may be empty) and bench.py arguments (no CPU
# baseline, no timing steps are added).  Prints "label round value ms_per_step" per run.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=${1:?out dir}; R=${2:?rounds}; shift 2
mkdir -p "$OUT"
for r in $(seq "$R"); do
  for v in "$@"; do
    IFS='|' read -r label envs args <<< "$v"
    log="$OUT/${label}_$r.log"
    # shellcheck disable=SC2086
    env $envs timeout -k 10 300 python bench.py --no-cpu-baseline --timing-steps 0 $args > "$log" 2>&1 \
      || { echo "$label $r FAILED"; tail -3 "$log"; exit 1; }
    echo "$label $r $(grep '^{' "$log" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
