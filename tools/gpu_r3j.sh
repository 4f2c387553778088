#!/bin/bash
# A/B: fence-light cross-stream waits (of_stream_wait) and the BN reductions on the side stream
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=${1:-gpurun_out/r3j}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_gpu_model.py tests/test_gpu_graph.py tests/test_gpu_dist.py > "$OUT/pytest.log" 2>&1
rc=$?
tail -2 "$OUT/pytest.log"
[ $rc -eq 0 ] || exit $rc
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > "$OUT/b_$tag.log" 2>&1 || { echo "bench $tag failed"; tail -5 "$OUT/b_$tag.log"; exit 1; }
  grep '^{' "$OUT/b_$tag.log" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', d['value'], d['ms_per_step'])"
}
for r in 1 2; do
  run new_$r OFLOW_X=1
  run torchwait_$r OFLOW_STREAM_WAIT=torch
  run bnmain_$r OFLOW_BN_SIDE=0
  run old_$r OFLOW_STREAM_WAIT=torch OFLOW_BN_SIDE=0
done
