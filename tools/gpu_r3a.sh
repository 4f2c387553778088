#!/bin/bash
# Round 3, first call: the new GPU tests (RCCL communicator, full-size parity, bf16
# teacher-forced modules), then the default bench with the full-batch CPU baseline.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=${1:-gpurun_out/r3a}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_bf16_modules.py \
  tests/test_gpu_fullsize.py -v -s --timeout 240 --timeout-method thread > "$OUT/pytest_new.log" 2>&1
rc=$?
grep -E "passed|failed|FAILED|ERROR|rel_l2|rel_inf|worst|loss hip|RCCL|cfg2:|192x640:" "$OUT/pytest_new.log" | tail -60
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 400 python bench.py > "$OUT/bench.log" 2>&1 || { echo bench failed; tail -5 "$OUT/bench.log"; exit 1; }
grep '^{' "$OUT/bench.log" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['frac'], d['cpu_baseline'], d['parity'])"
exit $rc
