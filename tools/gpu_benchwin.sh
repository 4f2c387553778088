#!/bin/bash
# Bench timing-window A/B: default (dominant kernel timed in the last 2 timed steps) vs no
# events in the timed region (--timing-steps 0) vs every conv timed (OFLOW_TIMING_DUMP set).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/benchwin
for r in 1 2; do
  for v in "def:" "none:--timing-steps 0" "all:DUMP"; do
    tag=${v%%:*}; a=${v#*:}
    if [ "$a" = "DUMP" ]; then
      out=$(OFLOW_TIMING_DUMP=/tmp/td.json timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline 2>/dev/null | grep '^{') || exit 1
    else
      out=$(timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline $a 2>/dev/null | grep '^{') || exit 1
    fi
    echo "$out" > gpurun_out/benchwin/$tag.$r.json
    echo "$tag $r: $(echo "$out" | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], d['ms_per_step'], (r or {}).get('kernel','')[11:50], (r or {}).get('frac'), (r or {}).get('avg_launch_ms'), (r or {}).get('launches_per_step'))")"
  done
done
