#!/bin/bash
# Interleaved A/B of the bench step: default vs. environment switches.
#   AB="ISG_NO_SIDE_FOLD=1;ISG_X=1 ISG_Y=1" tools/gpu_ab_env.sh TAG [rounds]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-ab}
A="--steps 100 --warmup 10 --no-cpu-baseline --no-infer --no-dense-leg --no-dp-leg"
IFS=';' read -ra VARS <<< "$AB"
for i in $(seq 1 ${2:-2}); do
  timeout -k 10 200 python -u bench.py $A > gpurun_out/ab_${TAG}_def_$i.log 2>&1 || exit 1
  grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_${TAG}_def_$i.log | sed "s/^/default $i /"
  j=0
  for v in "${VARS[@]}"; do
    j=$((j + 1))
    env $v timeout -k 10 200 python -u bench.py $A > gpurun_out/ab_${TAG}_v${j}_$i.log 2>&1 || exit 1
    grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_${TAG}_v${j}_$i.log | sed "s/^/$v $i /"
  done
done
