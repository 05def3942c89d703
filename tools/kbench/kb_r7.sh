#!/bin/bash
# round-5 stem kernels under the stamp build: phase medians per workgroup (kbench)
cd $GRAFT_REPO_ROOT/tools/kbench/_build
export KB_COEF=1
KB_STAMPS_DOWN=1 timeout -k 5 60 ./kbench fwd 2 16 512 512 16 5 2 2 1 200
KB_STAMPS_DOWN=1 timeout -k 5 60 ./kbench dgrad 2 16 512 512 16 5 2 2 1 200
KB_STAMPS_DOWN=1 timeout -k 5 60 ./kbench wgrad 2 16 512 512 16 5 2 2 1 200
KB_STAMPS_DOWN=1 timeout -k 5 60 ./kbench wgrad 2 3 1024 1024 16 5 2 2 1 200
KB_STAMPS_DOWN=1 timeout -k 5 60 ./kbench fwd 2 3 1024 1024 16 5 2 2 1 200
