#!/bin/bash
# Build the kbench harness in-tree: `build.sh` links it against the product libisg.so
# (timing only); `build.sh stamps` builds libisg_stamp.so (all kernels with -DISG_STAMPS,
# per-workgroup s_memrealtime stamps) and links against that instead.
set -e
cd "$(dirname "$0")"
if [ "${1:-}" != "stamps" ]; then
  mkdir -p _build
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O2 -std=c++17 kbench.cpp -o _build/kbench -ldl \
      -L../../instancesegmentation_amd -lisg -Wl,-rpath,'$ORIGIN/../../../instancesegmentation_amd'
  echo built _build/kbench "(libisg.so)"
  exit 0
fi
SRC=../../instancesegmentation_amd/csrc
OUT=$PWD/_build
mkdir -p $OUT
FL="--offload-arch=gfx950 -O2 -fno-unroll-loops -std=c++17 -fPIC -DISG_STAMPS -Wno-unused-function"
objs=""
for s in $SRC/*.hip; do
  f=$(basename $s .hip)
  /opt/rocm/bin/hipcc $FL -c $s -o $OUT/$f.o &
  objs="$objs $OUT/$f.o"
done
/opt/rocm/bin/hipcc $FL -x hip -c $SRC/api.cpp -o $OUT/api.o &
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/libisg_stamp.so $objs $OUT/api.o
/opt/rocm/bin/hipcc -O2 -std=c++17 kbench.cpp -o $OUT/kbench -ldl -L$OUT -lisg_stamp -Wl,-rpath,'$ORIGIN'
echo built $OUT/kbench
