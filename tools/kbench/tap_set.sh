#!/bin/bash
# fwd / dgrad shapes of the Segment(20) 1024^2 bs2 train step that run on tap_conv
cd "$(dirname "$0")/_build"
set -e
run() { timeout -k 5 60 ./kbench "$@"; }
run fwd 2 20 1024 1024 16 5 2 2 1     # init_conv.layer1 (stem)
run fwd 2 16 512 512 16 5 2 2 1       # init_conv.layer2
run dgrad 2 16 512 512 16 5 2 2 1     # dx init_conv.layer2
run fwd 2 4 1024 1024 1 3 1 1 1       # logits
run dgrad 2 4 1024 1024 1 3 1 1 1     # dx logits
run fwd 2 36 256 256 16 2 2 0 1       # bottle1_1.convs.0
run dgrad 2 36 256 256 16 2 2 0 1     # dx bottle1_1.convs.0
run fwd 2 16 128 128 16 3 1 1 1       # bottle4_3.convs.1
run dgrad 2 16 128 128 16 3 1 1 1
