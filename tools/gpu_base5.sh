#!/bin/bash
# Round-5 entry check: default bench (fp32 config 2) twice, bf16 B=32 once, with rocprof stats of the fp32 one.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=${1:-gpurun_out/base5}
mkdir -p "$OUT"
R="$GRAFT_REPO_ROOT/$OUT"
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; case $rc in 124|134|137|139) echo "step '$*' rc $rc: stopping"; exit $rc;; esac; return $rc; }
run 300 python bench.py --no-cpu-baseline > "$OUT/bench1.log" 2>&1 || { tail -5 "$OUT/bench1.log"; exit 1; }
grep '^{' "$OUT/bench1.log" | head -c 400; echo
run 300 python bench.py --no-cpu-baseline > "$OUT/bench2.log" 2>&1 || { tail -5 "$OUT/bench2.log"; exit 1; }
grep '^{' "$OUT/bench2.log" | head -c 400; echo
(cd /tmp && run 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/prof" -o bench -- \
  python "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline > "$R/bench_prof.log" 2>&1) || { echo rocprof failed; exit 1; }
run 300 python bench.py --precision bf16 --batch 32 --no-cpu-baseline > "$OUT/bench_bf16.log" 2>&1 || { tail -5 "$OUT/bench_bf16.log"; exit 1; }
grep '^{' "$OUT/bench_bf16.log" | head -c 300; echo
run 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_graph.py tests/test_gpu_dist.py "tests/test_gpu_model.py::test_resnet_block_bn_guard" "tests/test_gpu_model.py::test_bn_gamma_near_zero" "tests/test_gpu_model.py::test_two_forwards_one_backward" tests/test_gpu_bf16_modules.py -s > "$OUT/tests.log" 2>&1 || { echo tests failed; grep -E "^FAILED|Error" "$OUT/tests.log" | head; exit 1; }
tail -1 "$OUT/tests.log"
echo done
