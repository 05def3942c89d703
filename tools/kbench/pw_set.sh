#!/bin/bash
# 1x1 conv shapes of Segment(20) at bs2 1024^2 (slab kernels; "chunked" = the old ones).
# Usage: pw_set.sh [modes...]   (default: slab chunked). KB_COEF=1 is set: finalised BN
# coefficients, as in the training graph.
cd "$(dirname "$0")/_build"
export KB_COEF=1
modes=${@:-slab chunked}
for mode in $modes; do
  if [ $mode = chunked ]; then export ISG_PW_CHUNKED=1 ISG_PWG_OFF=1; else unset ISG_PW_CHUNKED ISG_PWG_OFF; fi
  echo "== $mode"
  for op in fwd dgrad wgrad; do
    for sh in "2 128 64 64 48" "2 48 64 64 128" "2 256 64 64 128" "2 48 128 128 16" "2 16 128 128 48" \
              "2 96 128 128 48" "2 36 256 256 16" "2 16 256 256 4"; do
      timeout -k 5 60 ./kbench $op $sh 1 1 0 1 200 || exit 1
    done
  done
done
