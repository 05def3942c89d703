#!/bin/bash
# kbench sweep: every shape under every environment setting.
#   SHAPES="op N Ci H W Co k s p d;..." ENVS="A=1 B=2;-;..." tools/gpu_sweep.sh TAG
# -> gpurun_out/sweep_TAG.log (one line per run: env, kbench line)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-x}
OUT=gpurun_out/sweep_$TAG.log
: > $OUT
IFS=';' read -ra SH <<< "$SHAPES"
IFS=';' read -ra EV <<< "$ENVS"
for s in "${SH[@]}"; do
  for e in "${EV[@]}"; do
    [ "$e" = "-" ] && e=""
    r=$(env $e timeout -k 5 30 tools/kbench/_build/kbench $s ${REPS:-50} 2>&1 | head -1) || { echo "FAIL [$e] $s: $r" | tee -a $OUT; exit 1; }
    echo "[$e] $r" | tee -a $OUT
  done
done
