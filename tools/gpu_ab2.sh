#!/bin/bash
# Interleaved A/B of the bench step over variants, each "ENV=V ENV2=V2 # --bench-flags"
# (either part may be empty; "-" alone = the default):
#   AB="-;ISG_SIDE_BATCH=16;# --eager;ISG_MAIN_PRIO=-1 # --eager" tools/gpu_ab2.sh TAG [rounds]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
TAG=${1:-ab}
A="--steps ${STEPS:-100} --warmup 10 --no-cpu-baseline --no-infer --no-dense-leg --no-dp-leg --no-roofline"
IFS=';' read -ra VARS <<< "$AB"
for i in $(seq 1 ${2:-2}); do
  j=0
  for v in "${VARS[@]}"; do
    j=$((j + 1))
    envs="${v%%#*}"; flags=""
    [[ "$v" == *"#"* ]] && flags="${v#*#}"
    [ "$envs" == "-" ] && envs=""
    env $envs timeout -k 10 200 python -u bench.py $A $flags > gpurun_out/ab_${TAG}_v${j}_$i.log 2>&1 \
        || { tail -5 gpurun_out/ab_${TAG}_v${j}_$i.log; exit 1; }
    echo "$v | round $i | $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_${TAG}_v${j}_$i.log)"
  done
done
