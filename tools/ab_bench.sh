#!/bin/bash
# GPU side of an A/B run of the whole step: bench.py (no CPU baseline) on the default library
# and on every tools/ab_build.sh variant, ROUNDS times interleaved (boxes differ by up to 10 %,
# so only same-call comparisons mean anything).   tools/ab_bench.sh [rounds] [steps]
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
R=${1:-2}; S=${2:-10}
for i in $(seq $R); do
  for d in base optical_flow_amd/_build/ab_*; do
    if [ "$d" = base ]; then lib=optical_flow_amd/liboflow.so; else lib=$d/liboflow.so; fi
    [ -f $lib ] || continue
    v=$(OFLOW_LIB=$lib timeout -k 10 200 python bench.py --steps $S --warmup 3 --no-cpu-baseline --timing-steps 0 2>/dev/null | grep '^{' | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])") || exit 1
    echo "$(basename $d) $v"
  done
done
