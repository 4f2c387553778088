#!/bin/bash
# Round-5 evidence in one GPU call: the whole -m gpu suite, smoke, FETCH_SIZE / WRITE_SIZE PMC
# passes for fp32 config 2, bf16 config 3 (B=32) and config 5 per GPU (768x1024 bf16 B=8), the
# default bench (fp32 config 2, CPU baseline on the bench batch) and its rocprofv3 kernel-trace
# summary, the bf16 benches and trace, the fp32-MFMA line, the flow / b16i micro-benchmarks.
# Publish with: bash tools/publish_round.sh gpurun_out/round5 r5
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=${1:-gpurun_out/round5}
mkdir -p "$OUT"
R="$GRAFT_REPO_ROOT/$OUT"
# a step that faulted, aborted, crashed or ran out of time ends the call
run() {
  local t=$1; shift
  timeout -k 10 "$t" "$@"; local rc=$?
  case $rc in 124|134|137|139) echo "step '$*' rc $rc: stopping"; exit $rc;; esac
  return $rc
}
run 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1 || { echo tests failed; grep -E "^FAILED|^ERROR" "$OUT/pytest_gpu.log" | head -10; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
run 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo smoke failed; tail -5 "$OUT/smoke.log"; exit 1; }
echo smoke ok
pmc() {   # $1 tag, rest: bench args
  local tag=$1; shift
  (cd /tmp && run 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/fetch_$tag" -o bench -- \
    python "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline "$@" > "$R/fetch_$tag.log" 2>&1) || { echo "fetch $tag failed"; return 1; }
  (cd /tmp && run 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/write_$tag" -o bench -- \
    python "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline "$@" > "$R/write_$tag.log" 2>&1) || { echo "write $tag failed"; return 1; }
}
pmc f32 || exit 1
python tools/pmc_traffic.py $OUT/fetch_f32/bench_counter_collection.csv $OUT/write_f32/bench_counter_collection.csv 384 512 8 fp32 > /dev/null || exit 1
pmc bf16 --precision bf16 --batch 32 || exit 1
python tools/pmc_traffic.py $OUT/fetch_bf16/bench_counter_collection.csv $OUT/write_bf16/bench_counter_collection.csv 384 512 32 bf16 > /dev/null || exit 1
pmc cfg5 --precision bf16 --height 768 --width 1024 --batch 8 || exit 1
python tools/pmc_traffic.py $OUT/fetch_cfg5/bench_counter_collection.csv $OUT/write_cfg5/bench_counter_collection.csv 768 1024 8 bf16 > /dev/null || exit 1
cp profiles/pmc_traffic.json $OUT/pmc_traffic.json
echo pmc ok
run 600 python bench.py > "$OUT/bench.log" 2>&1 || { echo bench failed; tail -5 "$OUT/bench.log"; exit 1; }
grep '^{' "$OUT/bench.log" | head -c 300; echo
# reproducibility: a second default run must end in the same timed_state (deterministic warp)
run 600 python bench.py --no-cpu-baseline > "$OUT/bench_repeat.log" 2>&1 || { echo bench repeat failed; exit 1; }
python - "$OUT/bench.log" "$OUT/bench_repeat.log" <<'PY' | tee "$OUT/timed_state_check.txt"
import json, sys
a, b = [json.loads([l for l in open(f) if l.startswith("{")][-1]) for f in sys.argv[1:3]]
print("timed_state identical:", a["timed_state"] == b["timed_state"], a["timed_state"]["last"])
PY
OFLOW_DETERMINISTIC=0 run 600 python bench.py --no-cpu-baseline > "$OUT/bench_atomic.log" 2>&1 || { echo atomic bench failed; exit 1; }
grep '^{' "$OUT/bench_atomic.log" | head -c 200; echo
(cd /tmp && run 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/prof" -o bench -- \
  python "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline > "$R/bench_prof.log" 2>&1) || { echo rocprof failed; exit 1; }
echo rocprof ok
run 600 python bench.py --precision bf16 --batch 32 --cpu-steps 1 > "$OUT/bench_bf16.log" 2>&1 || { echo bench bf16 failed; tail -5 "$OUT/bench_bf16.log"; exit 1; }
grep '^{' "$OUT/bench_bf16.log" | head -c 300; echo
(cd /tmp && run 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/prof_bf16" -o bench -- \
  python "$GRAFT_REPO_ROOT/bench.py" --precision bf16 --batch 32 --no-cpu-baseline > "$R/bench_bf16_prof.log" 2>&1) || { echo rocprof bf16 failed; exit 1; }
run 600 python bench.py --precision bf16 --height 768 --width 1024 --batch 8 --no-cpu-baseline > "$OUT/bench_cfg5.log" 2>&1 || { echo cfg5 bench failed; tail -5 "$OUT/bench_cfg5.log"; exit 1; }
grep '^{' "$OUT/bench_cfg5.log" | head -c 300; echo
OFLOW_F32_SPLIT=0 run 600 python bench.py --no-cpu-baseline > "$OUT/bench_f32mfma.log" 2>&1 || { echo f32mfma bench failed; exit 1; }
run 300 python tools/flow_bench.py --flow-scale 0.3 > "$OUT/flow_bench.txt" 2>&1 || { echo flow bench failed; exit 1; }
run 300 python tools/flow_bench.py --flow-scale 0.3 --flow-offset 21 > "$OUT/flow_bench_offset21.txt" 2>&1 || { echo flow bench failed; exit 1; }
run 300 python tools/b16i_bench.py --batch 32 > "$OUT/b16i_bench.txt" 2>&1 || { echo b16i bench failed; exit 1; }
echo done
