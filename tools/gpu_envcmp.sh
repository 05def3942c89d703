#!/bin/bash
# bench per-op tables under several environment settings: gpu_envcmp.sh TAG "ENV1" "ENV2" ...
cd "$GRAFT_REPO_ROOT"
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
TAG=$1; shift
i=0
for e in "$@"; do
  env $e timeout -k 10 200 python -u bench.py --steps ${STEPS:-20} --warmup 5 --no-cpu-baseline --no-infer \
      --no-dense-leg --profile-ops gpurun_out/ops_${TAG}_$i.txt > gpurun_out/bench_${TAG}_$i.log 2>&1 || exit 1
  echo "$i [$e] $(tail -1 gpurun_out/bench_${TAG}_$i.log | cut -c100-200)"
  i=$((i+1))
done
