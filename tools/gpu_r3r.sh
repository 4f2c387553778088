#!/bin/bash
# SQ counters of the bf16 3x3 kernels on dec3.c1 (B = 8): conv_tile_bf16 (key 12 = 0) and
# conv_tile_ws (key 12 = 2); one rocprofv3 --pmc pass each (8 SQ counters).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=${1:-gpurun_out/r3r}
mkdir -p "$OUT"
R="$GRAFT_REPO_ROOT/$OUT"
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
for t in 0 2; do
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d "$R/pmc_$t" -o cb -- \
    python "$GRAFT_REPO_ROOT/tools/conv_bench.py" --bf16 --reps 3 --only dec3.c1 --tune 12=$t > "$R/pmc_$t.log" 2>&1) || { echo "pmc $t failed"; tail -5 "$R/pmc_$t.log"; exit 1; }
done
echo done
