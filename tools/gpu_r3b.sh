#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=${1:-gpurun_out/r3b}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_bf16_modules.py "tests/test_gpu_fullsize.py::test_config2_384x512_b8_fp32" -v -s --timeout 240 --timeout-method thread > "$OUT/pytest_new.log" 2>&1
rc=$?
grep -E "passed|failed|FAILED|worst|cfg2:" "$OUT/pytest_new.log" | tail -30
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 400 python bench.py > "$OUT/bench.log" 2>&1 || { echo bench failed; tail -5 "$OUT/bench.log"; exit 1; }
grep '^{' "$OUT/bench.log" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['frac'], d['cpu_baseline'], d['parity'])"
exit $rc
