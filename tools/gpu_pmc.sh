#!/bin/bash
# PMC counters for the conv kernels of one layer shape (separate passes: the counter budget
# per pass is small on gfx950).
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=${1:-gpurun_out/pmc}
ONLY=${2:-dec3.c1}
mkdir -p "$OUT"
rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
i=0
for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_VMEM_WR" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d "$OUT/p$i" -o run -- \
    python tools/conv_bench.py --reps 3 --only "$ONLY" > "$OUT/p$i.log" 2>&1
  st=$?; echo "pass $i exit $st"; [ $st -ne 0 ] && { tail -5 "$OUT/p$i.log"; exit $st; }
done
exit 0
