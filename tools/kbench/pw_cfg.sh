#!/bin/bash
# (BM, BP) sweep of the pwx slab kernel over the Segment(20) 1x1 shapes (KB_COEF=1).
cd "$(dirname "$0")/_build"
export KB_COEF=1
for op in fwd dgrad; do
  for sh in "2 128 64 64 48" "2 48 64 64 128" "2 256 64 64 128" "2 48 128 128 16" "2 16 128 128 48" \
            "2 96 128 128 48" "2 36 256 256 16" "2 16 256 256 4"; do
    for bm in 16 32 48 64 96 128; do
      for bp in 16 32 64; do
        r=$(ISG_PWX_BM=$bm ISG_PWX_BP=$bp timeout -k 5 30 ./kbench $op $sh 1 1 0 1 100 2>&1 | head -1 | sed 's/.*: \([0-9.]*\) us.*/\1/')
        echo "$op [$sh] bm=$bm bp=$bp $r"
      done
    done
  done
done
