#!/bin/bash
cd $GRAFT_REPO_ROOT/tools/kbench/_build
export LD_LIBRARY_PATH=$GRAFT_REPO_ROOT/tools/kbench/stamplib:$LD_LIBRARY_PATH
export KB_COEF=1
timeout -k 5 60 ./kbench wgrad 2 48 64 64 128 1 1 0 1 200
timeout -k 5 60 ./kbench wgrad 2 128 64 64 48 1 1 0 1 200
timeout -k 5 60 ./kbench wgrad 2 16 128 128 48 1 1 0 1 200
timeout -k 5 60 ./kbench wgrad 2 48 128 128 16 1 1 0 1 200
