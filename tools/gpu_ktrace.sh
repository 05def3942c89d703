#!/bin/bash
# rocprofv3 kernel traces of a short bench run under several environment settings:
# gpu_ktrace.sh TAG "ENV1" "ENV2" ... -> gpurun_out/kt_TAG_i/ (analyse: tools/ktrace.py)
cd "$GRAFT_REPO_ROOT"
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
TAG=$1; shift
i=0
cd /tmp && export TMPDIR=/tmp
for e in "$@"; do
  ( export $e
  timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/kt_${TAG}_$i -o run --output-format csv \
      -- python3 $R/bench.py --steps ${STEPS:-20} --warmup 5 --no-cpu-baseline --no-infer --no-dense-leg ${BENCH_ARGS:-} \
      > $R/gpurun_out/kt_${TAG}_$i.log 2>&1 ) || exit 1
  echo "$i [$e] $(tail -1 $R/gpurun_out/kt_${TAG}_$i.log | cut -c100-200)"
  i=$((i+1))
done
