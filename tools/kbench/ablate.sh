#!/bin/bash
cd "$(dirname "$0")/_build"
for shape in "2 128 64 64 48 1 1 0 1" "2 16 128 128 48 1 1 0 1" "2 20 1024 1024 16 5 2 2 1"; do
 for d in 0 1 2 4 7; do
  echo "dbg=$d"; ISG_DBG=$d timeout -k 5 60 ./kbench wgrad $shape 20 | grep -E "^wgrad|seg"
 done
done
