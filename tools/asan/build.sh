#!/bin/bash
# Host-side AddressSanitizer build of every libisg source + the ABI driver:
#   tools/asan/build.sh [OUTDIR]   -> OUTDIR/abi_host_check (default tools/asan/_build)
# Device code is compiled normally (gfx950; GPU ASan is unavailable on this pool); only
# the host half is instrumented (-Xarch_host -fsanitize=address).
set -e
HERE=$(cd "$(dirname "$0")" && pwd)
ROOT=$(cd "$HERE/../.." && pwd)
OUT=${1:-$HERE/_build}
mkdir -p "$OUT"
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
# device code at -O0: the checks run without a GPU and never execute it (optimising the
# device half of every kernel took most of a 7-minute build; 3 minutes now)
FLAGS="--offload-arch=gfx950 -Xarch_host -fsanitize=address -Xarch_host -fno-omit-frame-pointer -Xarch_host -g -Xarch_host -O1 -Xarch_device -O0 -std=c++17"
objs=()
pids=()
for s in "$ROOT"/instancesegmentation_amd/csrc/*.hip "$ROOT"/instancesegmentation_amd/csrc/api.cpp \
         "$HERE/abi_host_check.cpp"; do
  o="$OUT/$(basename "${s%.*}").o"
  objs+=("$o")
  if [ -f "$o" ] && [ "$o" -nt "$s" ] && [ "$o" -nt "$ROOT/instancesegmentation_amd/csrc/common.h" ] \
     && [ "$o" -nt "$ROOT/instancesegmentation_amd/csrc/stage.h" ] && [ "$o" -nt "$ROOT/include/isg.h" ]; then
    continue
  fi
  lang=""; case "$s" in *.cpp) lang="-x hip";; esac
  $HIPCC $FLAGS $lang -c "$s" -o "$o" &
  pids+=($!)
done
for p in "${pids[@]}"; do wait "$p"; done
$HIPCC --offload-arch=gfx950 -Xarch_host -fsanitize=address -fno-gpu-sanitize -g "${objs[@]}" -o "$OUT/abi_host_check"
