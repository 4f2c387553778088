#!/bin/bash
# Round-6 evidence, part B (after part A, tools/gpu_round6a.sh, whose PMC file profiles/ must
# hold already): the
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
