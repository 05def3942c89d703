#!/bin/bash
# rocprofv3 kernel trace of the bench training leg alone under the given environment and
# bench flags:  ENVS="ISG_SIDE_BATCH=16" FLAGS="--eager" tools/gpu_trace_env.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out
TAG=${1:-t}
cd /tmp && export TMPDIR=/tmp
export $ENVS
timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/kt_$TAG -o run --output-format csv \
    -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-infer \
    --no-dense-leg --no-dp-leg --no-roofline $FLAGS \
    > $GRAFT_REPO_ROOT/gpurun_out/bench_kt_$TAG.log 2>&1 || { tail -30 $GRAFT_REPO_ROOT/gpurun_out/bench_kt_$TAG.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*' $GRAFT_REPO_ROOT/gpurun_out/bench_kt_$TAG.log
