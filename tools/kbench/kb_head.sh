#!/bin/bash
# mask-head kernels under the stamp build: per-workgroup phase medians (kbench)
cd $GRAFT_REPO_ROOT/tools/kbench/_build
KB_STAMPS=isg_dbg_stamps_head timeout -k 5 60 ./kbench headb 2 16 256 256 16 1 1 0 1 200
KB_STAMPS=isg_dbg_stamps_head timeout -k 5 60 ./kbench headf 2 16 256 256 16 1 1 0 1 200
