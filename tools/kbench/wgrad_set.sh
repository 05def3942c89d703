#!/bin/bash
# wgrad shapes of the Segment(20) 1024^2 bs2 train step (tools/plan_dump.py)
cd "$(dirname "$0")/_build"
set -e
run() { timeout -k 5 60 ./kbench wgrad "$@"; }
run 2 128 64 64 48 1 1 0 1      # bottle2_x.*.convs.0
run 2 48 64 64 128 1 1 0 1      # bottle2_x.*.convs.2
run 2 256 64 64 128 1 1 0 1     # bottle3_1.resconv
run 2 48 128 128 16 1 1 0 1     # bottle1_x.*.convs.0
run 2 16 128 128 48 1 1 0 1     # bottle1_x.*.convs.2
run 2 96 128 128 48 1 1 0 1     # bottle4_2.resconv
run 2 16 128 128 16 3 1 1 1     # bottle4_3.convs.1 (dense 3x3)
run 2 4 256 256 4 3 1 1 1       # bottle5_2.convs.1
run 2 36 256 256 16 2 2 0 1     # bottle1_1.convs.0 (2x2 s2)
run 2 16 512 512 16 5 2 2 1     # init_conv.layer2
run 2 20 1024 1024 16 5 2 2 1   # init_conv.layer1 (stem)
run 2 4 1024 1024 1 3 1 1 1     # logits
