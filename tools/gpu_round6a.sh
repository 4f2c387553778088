#!/bin/bash
# Round-6 evidence, part A (tests, smoke, PMC passes): the whole -m gpu suite, smoke, FETCH_SIZE / WRITE_SIZE PMC
# passes for fp32 config 2, bf16 config 3 (B=32) and config 5 per GPU (768x1024 bf16 B=8), the
# default bench (fp32 config 2, CPU baseline on the bench batch) and its rocprofv3 kernel-trace
# summary, the bf16 benches and trace, the fp32-MFMA line, the flow / b16i micro-benchmarks.
# Round 6 adds an MFMA-utilisation PMC pass per configuration (SQ_VALU_MFMA_BUSY_CYCLES,
# SQ_BUSY_CYCLES, GRBM_GUI_ACTIVE; tools/pmc_mfma.py merges it into profiles/pmc_traffic.json,
# which the benches then read: roofline.mfma_busy).
# Publish with: bash tools/publish_round.sh gpurun_out/round6 r6
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=${1:-gpurun_out/round6}
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
  (cd /tmp && run 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$R/mfma_$tag" -o bench -- \
    python "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline "$@" > "$R/mfma_$tag.log" 2>&1) || { echo "mfma $tag failed"; return 1; }
}
pmc f32 || exit 1
python tools/pmc_traffic.py $OUT/fetch_f32/bench_counter_collection.csv $OUT/write_f32/bench_counter_collection.csv 384 512 8 fp32 > /dev/null || exit 1
python tools/pmc_mfma.py $OUT/mfma_f32/bench_counter_collection.csv 384 512 8 fp32 > $OUT/mfma_f32.md || exit 1
pmc bf16 --precision bf16 --batch 32 || exit 1
python tools/pmc_traffic.py $OUT/fetch_bf16/bench_counter_collection.csv $OUT/write_bf16/bench_counter_collection.csv 384 512 32 bf16 > /dev/null || exit 1
python tools/pmc_mfma.py $OUT/mfma_bf16/bench_counter_collection.csv 384 512 32 bf16 > $OUT/mfma_bf16.md || exit 1
pmc cfg5 --precision bf16 --height 768 --width 1024 --batch 8 || exit 1
python tools/pmc_traffic.py $OUT/fetch_cfg5/bench_counter_collection.csv $OUT/write_cfg5/bench_counter_collection.csv 768 1024 8 bf16 > /dev/null || exit 1
python tools/pmc_mfma.py $OUT/mfma_cfg5/bench_counter_collection.csv 768 1024 8 bf16 > $OUT/mfma_cfg5.md || exit 1
cp profiles/pmc_traffic.json $OUT/pmc_traffic.json
echo pmc ok
echo partA done
