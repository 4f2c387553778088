#!/bin/bash
# fp32 B=8 A/B of the round-2-end tree (12eca7a, built in _abprev/) against the current tree,
# alternating on one box.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=$PWD/gpurun_out/r3u
mkdir -p "$OUT"
for r in 1 2 3; do
  (cd _abprev && timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > "$OUT/prev_$r.log" 2>&1) || { echo prev failed; tail -3 "$OUT/prev_$r.log"; exit 1; }
  echo "prev $r $(grep -o '"value": [0-9.]*' $OUT/prev_$r.log)"
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > "$OUT/cur_$r.log" 2>&1 || { echo cur failed; tail -3 "$OUT/cur_$r.log"; exit 1; }
  echo "cur  $r $(grep -o '"value": [0-9.]*' $OUT/cur_$r.log)"
done
