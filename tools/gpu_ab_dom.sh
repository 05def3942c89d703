#!/bin/bash
# per-op pass before capture vs none: does the per-op pass slow the timed step?
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
A="--steps 100 --warmup 10 --no-cpu-baseline --no-infer --no-dense-leg --no-dp-leg"
for i in 1 2; do
  timeout -k 10 200 python -u bench.py $A > gpurun_out/abd_def_$i.log 2>&1 || exit 1
  grep -o '"ms_per_step": [0-9.]*' gpurun_out/abd_def_$i.log | sed "s/^/default $i /"
  timeout -k 10 200 python -u bench.py $A --dominant bwd:d_out0 > gpurun_out/abd_dom_$i.log 2>&1 || exit 1
  grep -o '"ms_per_step": [0-9.]*' gpurun_out/abd_dom_$i.log | sed "s/^/dominant $i /"
done
