#!/bin/bash
# Build an experimental variant of libisg.so with extra preprocessor definitions:
#   tools/build_variant.sh NAME "-DISG_STAT_REP=4 ..."  -> instancesegmentation_amd/libisg_NAME.so
# Select it at run time with ISG_LIB=<path> (plus ISG_STAT_REP=<n> when the count changes).
set -e
cd "$(dirname "$0")/.."
NAME=$1; DEFS=$2
SRC=instancesegmentation_amd/csrc
OUT=instancesegmentation_amd/build_obj_$NAME
mkdir -p $OUT
FL="--offload-arch=gfx950 -O2 -fno-unroll-loops -std=c++17 -fPIC -Wno-unused-function -Wno-pass-failed $DEFS"
objs=""
for s in $SRC/*.hip; do
  f=$(basename $s .hip)
  /opt/rocm/bin/hipcc $FL -c $s -o $OUT/$f.o &
  objs="$objs $OUT/$f.o"
  while [ $(jobs -r | wc -l) -ge 6 ]; do sleep 1; done
done
/opt/rocm/bin/hipcc $FL -x hip -c $SRC/api.cpp -o $OUT/api.o
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o instancesegmentation_amd/libisg_$NAME.so $objs $OUT/api.o
echo built instancesegmentation_amd/libisg_$NAME.so
