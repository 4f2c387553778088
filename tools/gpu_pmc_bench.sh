#!/bin/bash
# FETCH_SIZE and WRITE_SIZE passes (separate, per the guide) over the default bench command.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=${1:-gpurun_out/pmcb}
mkdir -p "$OUT"
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o bench -- \
  python bench.py --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/fetch.log" 2>&1
st=$?; echo "fetch pass $st"; [ $st -ne 0 ] && exit $st
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o bench -- \
  python bench.py --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/write.log" 2>&1
st=$?; echo "write pass $st"; exit $st
