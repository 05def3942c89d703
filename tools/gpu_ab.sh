#!/bin/bash
# Interleaved A/B of the captured train step under environment settings:
#   gpu_ab.sh TAG REPS "ENV_A" "ENV_B" ...   (each ENV a space-separated VAR=val list, "-" = none)
# -> one line per run: setting index, images/s, ms/step (bench.py, no per-op pass).
cd "$GRAFT_REPO_ROOT"
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
TAG=$1; REPS=$2; shift 2
for r in $(seq 1 $REPS); do
  i=0
  for e in "$@"; do
    [ "$e" = "-" ] && e=""
    env $e timeout -k 10 200 python -u bench.py --steps ${STEPS:-200} --warmup 10 --no-cpu-baseline \
        --no-infer --no-dense-leg --no-roofline ${BENCH_ARGS:-} > gpurun_out/ab_${TAG}_${i}_$r.log 2>&1 || { tail -20 gpurun_out/ab_${TAG}_${i}_$r.log; exit 1; }
    python - gpurun_out/ab_${TAG}_${i}_$r.log "$i" "$e" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], f"{d['value']:.1f} img/s {d['ms_per_step']:.3f} ms", sys.argv[3] or "(default)", flush=True)
PY
    i=$((i+1))
  done
done
