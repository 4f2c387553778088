#!/bin/bash
# PMC passes over tools/flow_bench.py (level-3 cost-volume / warp kernels): HBM bytes and SQ
# issue counters per kernel.  Summarise with tools/pmc_summary.py-style grouping by hand.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=${1:-gpurun_out/pmc_flow4}
R="$GRAFT_REPO_ROOT/$OUT"
mkdir -p "$OUT"
p() {
  local tag=$1; shift
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d "$R/$tag" -o fb -- \
    python "$GRAFT_REPO_ROOT/tools/flow_bench.py" --flow-scale 0.3 --reps 3 > "$R/$tag.log" 2>&1) || { echo "$tag failed"; exit 1; }
  echo "$tag ok"
}
p fetch FETCH_SIZE
p write WRITE_SIZE
p sq SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT
