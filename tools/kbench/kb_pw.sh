#!/bin/bash
# the 64^2 block's 1x1 kernels under the stamp build: per-workgroup phase medians (kbench)
cd $GRAFT_REPO_ROOT/tools/kbench/_build
export KB_COEF=1
for op in fwd dgrad; do
  timeout -k 5 60 ./kbench $op 2 48 64 64 128 1 1 0 1 200
  timeout -k 5 60 ./kbench $op 2 128 64 64 48 1 1 0 1 200
done
timeout -k 5 60 ./kbench wgrad 2 48 64 64 128 1 1 0 1 200
