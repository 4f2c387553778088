#!/bin/bash
# PMC counter passes (one rocprofv3 run per counter set) over an arbitrary python command.
# Usage: tools/gpu_pmc_cmd.sh OUTDIR python tools/flow_bench.py --reps 2
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=$1; shift
mkdir -p "$OUT"
i=0
for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_VMEM_WR" \
           "SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d "$OUT/p$i" -o run -- \
    "$@" > "$OUT/p$i.log" 2>&1
  st=$?; echo "pass $i exit $st"; [ $st -ne 0 ] && { tail -5 "$OUT/p$i.log"; exit $st; }
done
exit 0
